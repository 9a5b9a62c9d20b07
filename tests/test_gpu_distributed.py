"""The sharded multi-GPU paths on the GPU, rehearsed on the one card of the test box: two
processes (world_size 2, gloo over the host for the collectives; the real runs use one GPU
per rank and RCCL) each run the HIP kernels on their own shard.

* configs[2] (bench.py's workload): contiguous blocks of global ray ids, forward-tree roots
  sampled by the GPU sampler (Philox keyed by the global ray id), RT.propagate, the binned
  flux and its all-reduce. Every per-ray output of a shard equals the same rays of the
  single-process run bit for bit, and the reduced flux and totals equal the single-process
  ones exactly (integer-valued counts).
* main_runner_tree sharded by global event id: the ranks' npy rows in rank
  order equal the single-process rows, column 8 divided by the GLOBAL f_inx
  (MainRunner.jl:747), and the reduced radiated flux equals the single-process one.
* the device binned flux equals plot/flux.py's np.histogram over the written rows.
* the C-ABI reduction (art_comm_* / art_flux_allreduce, RCCL) on a world of one.
"""
import os
import socket

import numpy as np
import pytest

from conftest import CONFIGS

pytestmark = pytest.mark.gpu

N_RAYS = 20_000
NBINS = 50
N_TRAJS = 41  # 40 events


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _segments(lo, hi, kw):
    import torch
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    eng = Engine(A.Params(**kw), device=0)
    inp = eng.forward_roots(hi - lo, seed=1769, ray_offset=lo)
    out = eng.propagate(inp, max_crossings=-1)
    hist = eng.flux_histogram(out, inp["species"], None, NBINS)
    torch.cuda.synchronize()
    keys = ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept", "n_reject", "n_cross", "xc_pos", "xc_p")
    return {k: out[k].cpu().numpy() for k in keys}, hist, int(out["n_accept"].sum().item())


def _worker(rank, world, port, kw, outdir, what):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if what == "segments":
            from adiabatic_raytracer_amd.shard import allreduce_flux, reduce_totals, shard_range
            lo, hi = shard_range(N_RAYS, rank, world)
            o, hist, steps = _segments(lo, hi, kw)
            h = hist.cpu()
            allreduce_flux(h, world)
            tot_steps, _, tot_rays = reduce_totals(steps, 1.0, hi - lo, world)
            np.savez(os.path.join(outdir, f"seg{rank}.npz"), hist=h.numpy(), steps=tot_steps, rays=tot_rays, lo=lo,
                     hi=hi, **o)
        else:
            import adiabatic_raytracer_amd as A
            info = {}
            A.trees.main_runner_tree(A.Params(**kw), N_TRAJS, saveMode=1, dir_tag=outdir, file_tag="s", rank=rank,
                                     world=world, run_info=info)
            np.savez(os.path.join(outdir, f"ev{rank}.npz"), flux=info["flux"], f_inx=info["f_inx"],
                     rows=info["rows"], sw=np.asarray(info["sum_weight_sln_prob"]))
    finally:
        dist.destroy_process_group()


def _spawn(kw, tmp_path, what):
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(2, _free_port(), kw, str(tmp_path), what), nprocs=2, join=True,
                       start_method="spawn")


def test_configs2_segment_shards_match_single_process(tmp_path):
    kw = CONFIGS["flat"]
    _spawn(kw, tmp_path, "segments")
    full, hist, steps = _segments(0, N_RAYS, kw)
    h_full = hist.cpu().numpy()
    n = N_RAYS
    for r in range(2):
        z = np.load(tmp_path / f"seg{r}.npz")
        assert np.array_equal(z["hist"], h_full)  # exact: integer-valued counts
        assert int(z["steps"]) == steps and int(z["rays"]) == n
        lo, hi = int(z["lo"]), int(z["hi"])
        m = hi - lo
        for k in ("u7_end", "tau_end", "status", "n_accept", "n_reject", "n_cross", "xc_p"):
            assert np.array_equal(z[k], full[k][lo:hi], equal_nan=True), k  # (NaN: no crossing)
        for k in ("x_end", "k_end", "xc_pos"):
            assert np.array_equal(z[k].reshape(3, m), full[k].reshape(3, n)[:, lo:hi], equal_nan=True), k
    assert h_full[NBINS:].sum() > 0


def test_event_shards_match_single_process(tmp_path):
    import adiabatic_raytracer_amd as A
    kw = CONFIGS["flat"]
    _spawn(kw, tmp_path, "events")
    p = A.Params(**kw)
    info = {}
    rows = A.trees.main_runner_tree(p, N_TRAJS, saveMode=1, run_info=info)
    both = A.trees.gather_rank_rows(str(tmp_path), p, N_TRAJS, 2, file_tag="s")
    # rows: global event ids, the global f_inx in column 8 -- the single-process file
    assert both.shape == rows.shape and np.array_equal(both[:, 0], rows[:, 0])
    assert np.array_equal(both, rows, equal_nan=True)  # bit for bit
    for r in range(2):
        z = np.load(tmp_path / f"ev{r}.npz")
        assert int(z["f_inx"]) == info["f_inx"] and int(z["rows"]) == len(rows)
        np.testing.assert_allclose(z["flux"], info["flux"], rtol=1e-12, atol=0)
        np.testing.assert_allclose(z["sw"], info["sum_weight_sln_prob"], rtol=1e-12, atol=0)
    # the npy files carry file_tag + rank (MainRunner.jl:750-761)
    names = sorted(f.name for f in (tmp_path / "npy").glob("tree_*.npy"))
    assert len(names) == 2 and names[0].endswith("_s0.npy") and names[1].endswith("_s1.npy")


def test_radiated_flux_is_flux_py_histogram(tmp_path):
    """plot/flux.py:38-48: np.histogram(phif, 50, weights=weight*sln_prob*(id==1)) over the
    written rows, with the build's fixed range (-π, π)."""
    import adiabatic_raytracer_amd as A
    p = A.Params(**CONFIGS["flat"])
    info = {}
    rows = A.trees.main_runner_tree(p, 201, saveMode=0, dir_tag=str(tmp_path), file_tag="f", run_info=info)
    res = np.load(next((tmp_path / "npy").glob("tree_*.npy")))
    assert np.array_equal(res, rows, equal_nan=True)
    particle_id, phif, sln_prob, weight = res[:, 1].astype(int), res[:, 3], res[:, 7], res[:, 8]
    pps = weight * sln_prob
    for row, ident in ((1, 1), (0, 0)):
        ref, edges = np.histogram(phif, bins=NBINS, range=(-np.pi, np.pi), weights=pps * (particle_id == ident))
        np.testing.assert_allclose(info["flux"][row], ref, rtol=1e-12, atol=1e-300)
    assert info["flux"][1].sum() > 0
    # the device binning is numpy's, bin for bin, including values on the edges
    edges = np.linspace(-np.pi, np.pi, NBINS + 1)
    phi = np.concatenate([edges, np.nextafter(edges, 3.0), np.nextafter(edges, -3.0), [np.nan, 3.2, -3.2]])
    h = A.trees.radiated_flux(phi, np.ones(phi.size), np.arange(1.0, phi.size + 1.0), NBINS)
    ref = np.histogram(phi, bins=NBINS, range=(-np.pi, np.pi), weights=np.arange(1.0, phi.size + 1.0))[0]
    assert np.array_equal(h[NBINS:], ref) and not h[:NBINS].any()


def test_capi_flux_allreduce_world1():
    """art_comm_unique_id / art_comm_init / art_flux_allreduce / art_comm_destroy through
    ctypes: the reduction a Julia host driving one process per GPU would call
    (INTEGRATION.md). On a world of one the sum is the identity."""
    import ctypes as C
    import torch
    import adiabatic_raytracer_amd as A
    lib = A._lib.load()
    torch.cuda.set_device(0)
    A._lib.check(lib.art_set_device(0))
    uid = (C.c_char * 128)()
    A._lib.check(lib.art_comm_unique_id(uid))
    A._lib.check(lib.art_comm_init(0, 1, uid))
    try:
        h = torch.arange(100, dtype=torch.float64, device="cuda") * 0.5
        ref = h.clone()
        A._lib.check(lib.art_flux_allreduce(C.c_void_p(h.data_ptr()), h.numel(),
                                            C.c_void_p(torch.cuda.current_stream().cuda_stream)))
        torch.cuda.synchronize()
        assert torch.equal(h, ref)
        hh = np.arange(7, dtype=np.float64)
        A._lib.check(lib.art_flux_allreduce_host(hh.ctypes.data_as(C.c_void_p), hh.size))
        assert np.array_equal(hh, np.arange(7.0))
    finally:
        A._lib.check(lib.art_comm_destroy())
