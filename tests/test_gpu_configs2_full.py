"""BASELINE.json configs[2] at its own size: the 10^7-ray GJ-dipole batch, sharded by
contiguous global ray ids over one process per rank, with the binned flux all-reduced
(the reference's process fan-out is runner_example.sh:4-7 and its merge
Gen_Samples.jl:195-239 / Combine_Files.py). On the one-GPU test box every rank runs on the
same card and the collectives go over gloo (the real runs: one GPU per rank, RCCL).

* world 2 (5e6 rays per rank) and world 8 (1.25e6 per rank, the 8-GPU split): every per-ray
  output of every shard equals the same rays of the single-process 10^7-ray run bit for bit
  (compared through SHA-256 digests of each SoA row, so no rank ships 0.5 GB back), the
  all-reduced flux histogram and the run's totals (Σ accepted steps, Σ rays) equal the
  single-process ones exactly (integer-valued sums);
* a 512-ray slice from the middle of each world-2 shard is held to the oracle on the same
  initial conditions with test_gpu_propagate's 1-ulp envelope (_compare);
* bench.py's own N > 1 path (torch.distributed.run, two ranks, gloo rehearsal on the one
  card) prints one line whose totals are the sum over the shards.
"""
import hashlib
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import CONFIGS

pytestmark = pytest.mark.gpu

N_RAYS = 10_000_000
NBINS = 50
SLICE = 512
KEYS = ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept", "n_reject", "n_cross", "xc_pos", "xc_k", "xc_t",
        "xc_dw", "xc_p")
VEC = ("x_end", "k_end", "xc_pos", "xc_k")  # 3 SoA rows each (capacity 1)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _digest(t):
    return hashlib.sha256(t.contiguous().cpu().numpy().tobytes()).hexdigest()


def _row_digests(out, m, lo=0, hi=None):
    """SHA-256 of every SoA row of the outputs over rays [lo, hi) of a batch of m rays."""
    hi = m if hi is None else hi
    d = {}
    for k in KEYS:
        if k in VEC:
            v = out[k].view(3, m)
            for c in range(3):
                d[f"{k}{c}"] = _digest(v[c, lo:hi])
        else:
            d[k] = _digest(out[k][lo:hi])
    return d


def _run_shard(lo, hi, kw):
    """Sample the forward-tree roots of global rays [lo, hi) on the GPU and propagate them."""
    import torch
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    eng = Engine(A.Params(**kw), device=0)
    inp = eng.forward_roots(hi - lo, seed=1769, ray_offset=lo)
    out = eng.propagate(inp, max_crossings=-1)
    hist = eng.flux_histogram(out, inp["species"], None, NBINS)
    torch.cuda.synchronize()
    return inp, out, hist


def _slice_npz(inp, out, m, a, b):
    """Inputs and outputs of rays [a, b) of a batch of m rays, in the SoA layout of
    oracle.propagate / raytracer.propagate_batch."""
    z = {}
    for k in ("x0", "k0"):
        z[k] = inp[k].view(3, m)[:, a:b].cpu().numpy().reshape(-1)
    z["erg"] = inp["erg"][a:b].cpu().numpy()
    for k in KEYS:
        z[k] = (out[k].view(3, m)[:, a:b] if k in VEC else out[k][a:b]).cpu().numpy().reshape(-1)
    return z


def _worker(rank, world, port, kw, outdir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from adiabatic_raytracer_amd.shard import allreduce_flux, reduce_totals, shard_range
        lo, hi = shard_range(N_RAYS, rank, world)
        m = hi - lo
        inp, out, hist = _run_shard(lo, hi, kw)
        steps = int(out["n_accept"].sum().item())
        h = hist.cpu()
        allreduce_flux(h, world)  # bench.py's collective
        tot_steps, _, tot_rays = reduce_totals(steps, 1.0, m, world)
        res = {"lo": lo, "hi": hi, "hist": h.numpy().tolist(), "steps": tot_steps, "rays": tot_rays,
               "digests": _row_digests(out, m)}
        with open(os.path.join(outdir, f"shard{world}_{rank}.json"), "w") as f:
            json.dump(res, f)
        if world == 2:  # the slice for the oracle check: the middle of the shard
            a = m // 2
            np.savez(os.path.join(outdir, f"slice{rank}.npz"), lo=lo + a, **_slice_npz(inp, out, m, a, a + SLICE))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def single_process():
    """The single-process 10^7-ray run: flux, totals and the digests of every shard's rays for
    world 2 and world 8."""
    from adiabatic_raytracer_amd.shard import shard_range
    inp, out, hist = _run_shard(0, N_RAYS, CONFIGS["flat"])
    res = {"hist": hist.cpu().numpy(), "steps": int(out["n_accept"].sum().item()), "digests": {}}
    for world in (2, 8):
        for r in range(world):
            lo, hi = shard_range(N_RAYS, r, world)
            res["digests"][(world, r)] = _row_digests(out, N_RAYS, lo, hi)
    res["status"] = np.bincount(out["status"].cpu().numpy(), minlength=5)
    del inp, out
    import torch
    torch.cuda.empty_cache()
    return res


@pytest.mark.parametrize("world", [2, 8])
def test_configs2_full_size_shards(world, single_process, tmp_path, oracle_lib):
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(world, _free_port(), CONFIGS["flat"], str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    ref = single_process
    assert ref["status"][1] > 1e6 and ref["hist"][NBINS:].sum() > 1e6  # crossings and escaping photons both present
    covered = 0
    for r in range(world):
        z = json.load(open(tmp_path / f"shard{world}_{r}.json"))
        covered += z["hi"] - z["lo"]
        # the all-reduced flux and the totals: exact (integer-valued sums of 1.0 and counts)
        assert np.array_equal(np.asarray(z["hist"]), ref["hist"]), r
        assert int(z["steps"]) == ref["steps"] and int(z["rays"]) == N_RAYS, (z["steps"], ref["steps"])
        want = ref["digests"][(world, r)]
        bad = [k for k in want if z["digests"][k] != want[k]]
        assert not bad, (world, r, bad)  # every per-ray output row bit for bit
    assert covered == N_RAYS
    if world != 2:
        return
    # the middle 512 rays of each world-2 shard (the sharded run's own outputs) against the
    # oracle on the same initial conditions, with test_gpu_propagate's 1-ulp envelope
    from test_gpu_propagate import N_PERTURB, _compare
    po = oracle_lib.make_params(**CONFIGS["flat"])
    for r in range(2):
        z = dict(np.load(tmp_path / f"slice{r}.npz"))
        n = z["erg"].size
        assert n == SLICE
        sp = np.ones(n, np.int8)
        o = oracle_lib.propagate(po, z["x0"], z["k0"], z["erg"], -1.0, -30.0, sp, max_crossings=-1, cap=1)
        o2 = []
        for k in range(N_PERTURB):
            ulp = np.random.default_rng(1769 + k).choice([-1.0, 1.0], z["x0"].shape) * 2.2e-16
            o2.append(oracle_lib.propagate(po, z["x0"] * (1.0 + ulp), z["k0"], z["erg"], -1.0, -30.0, sp,
                                           max_crossings=-1, cap=1))
        _compare(z, o, o2, n)


def test_bench_two_rank_rehearsal():
    """bench.py --gpus 2 under torch.distributed.run (both ranks on the one card, gloo): rank 0
    prints one JSON line whose rays and ray-steps are the whole job's."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ART_BENCH_DEVICE="0", ART_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(root, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--rays", "400000", "--no-cpu-baseline", "--no-pcie"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["steps"] == 2
    assert line["config"]["workload"].startswith("400000 ")
