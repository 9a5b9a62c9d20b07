"""Host logic of the parameter scan (BASELINE.json configs[4], adiabatic_raytracer_amd/scan.py)
and of the reference's Julia combine step (Gen_Samples.jl:195-239, trees.combine_files)."""
import os
import socket

import numpy as np
import pytest


def test_scan_grid_is_the_baseline_grid():
    from adiabatic_raytracer_amd.scan import scan_grid
    g = scan_grid()
    assert len(g) == 32
    assert {p["mass_a"] for p in g} == {1e-6, 2e-6, 5e-6, 1e-5}
    assert {p["B0"] for p in g} == {2.5e13, 5e13, 1e14, 2e14}
    assert sorted({round(2 * np.pi / p["omega_pul"], 12) for p in g}) == [0.5, 1.0]


def test_points_partition():
    from adiabatic_raytracer_amd.scan import points_of_rank
    for world in (1, 2, 3, 8):
        got = sorted(i for r in range(world) for i in points_of_rank(32, r, world))
        assert got == list(range(32))
        sizes = [len(points_of_rank(32, r, world)) for r in range(world)]
        assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        points_of_rank(32, 2, 2)


def test_every_grid_point_has_a_conversion_surface():
    """all 32 points have maxR in [29.3, 342] km > rNS."""
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd.scan import scan_grid
    r = [A.Find_Conversion_Surface(A.Params(**kw)) for kw in scan_grid()]
    assert min(r) > 10.0 and 25.0 < min(r) and max(r) < 400.0, (min(r), max(r))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fake_run(kw, rays, seed, device=0):
    return {"mass_a": kw["mass_a"], "B0": kw["B0"], "rays": rays, "seed": seed}


def _worker(rank, world, port, outdir):
    import json
    import torch.distributed as dist
    from adiabatic_raytracer_amd.scan import run_scan
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        recs = run_scan(7, None, 1769, run=_fake_run)
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as fh:
            json.dump(recs, fh)
    finally:
        dist.destroy_process_group()


def test_scan_gather_world2(tmp_path):
    """Two gloo ranks split the 32 points and both end with all 32 records in grid order."""
    import json
    import torch.multiprocessing as mp
    from adiabatic_raytracer_amd.scan import scan_grid
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    g = scan_grid()
    for r in range(2):
        recs = json.load(open(tmp_path / f"r{r}.json"))
        assert [x["point"] for x in recs] == list(range(32))
        assert all(x["mass_a"] == g[x["point"]]["mass_a"] and x["B0"] == g[x["point"]]["B0"] for x in recs)


def test_combine_files_matches_gen_samples(tmp_path):
    """combine_files: vcat of the per-run npy files, 1-based column 8 divided by Nruns, inputs removed."""
    from adiabatic_raytracer_amd.trees import combine_files, tree_file_name
    args = (1e-5, 1e-12, 0.2, 1.0, 1e14)
    rng = np.random.default_rng(0)
    parts = []
    for i in range(3):
        f = tree_file_name(str(tmp_path), *args, 100, 3, 5, 5, 50, f"run{i}")
        os.makedirs(os.path.dirname(f), exist_ok=True)
        a = rng.normal(size=(4 + i, 13))
        np.save(f, a)
        parts.append(a)
    out = combine_files(*args, 100, 3, "run", dir_tag=str(tmp_path))
    want = np.concatenate(parts)
    want[:, 7] /= 3
    assert os.path.basename(out) == "MassAx_1.0e-5_AxionG_1.0e-12_ThetaM_0.2_rotPulsar_1.0_B0_1.0e14_Ax_trajs_300" \
                                    "_N_Times_3_num_cutoff_5_MC_nodes_5_max_nodes_50_run.npy"
    assert np.array_equal(np.load(out), want)
    assert not list((tmp_path / "npy").glob("*.npy"))
