"""Multi-GPU path on CPU: world_size-2 `gloo` run of the sharding and reductions that
bench.py uses (adiabatic_raytracer_amd/shard.py). Each rank samples its contiguous
block of global ray ids (Philox keyed by the global id), propagates it with the oracle
(CPU stand-in for the GPU kernel, test-only), bins the escaping photons as flux_kernel
does (plot/flux.py:38-48 with a fixed [-pi, pi) range) and all-reduces. The reduced
histogram and totals must equal the single-process result on the whole batch."""
import os
import socket

import numpy as np
import pytest

from conftest import CONFIGS

N_RAYS = 48
NBINS = 50


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _flux_hist(o, n, nbins=NBINS, rns=10.0):
    """Host restatement of flux_kernel: photons that ended without a crossing beyond 1.1 rNS,
    binned by atan2(k_y, k_x) as np.histogram(range=(-pi, pi))."""
    x, k = o["x_end"].reshape(3, n), o["k_end"].reshape(3, n)
    keep = (o["status"] != 1) & (np.linalg.norm(x, axis=0) > 1.1 * rns)
    phi = np.arctan2(k[1], k[0])
    h = np.zeros(2 * nbins)
    h[nbins:] = np.histogram(phi[keep], nbins, range=(-np.pi, np.pi))[0]
    return h


def _shard_work(rank, world, n_total, kw):
    import oracle as O
    from adiabatic_raytracer_amd.shard import shard_range
    lo, hi = shard_range(n_total, rank, world)
    po = O.make_params(**kw)
    s = O.sample(po, O.find_conversion_surface(po), 1769, lo, hi - lo)
    o = O.propagate(po, s["x"], s["k_init"], s["erg"], -1.0, -30.0, 1, max_crossings=-1, nthreads=2)
    return _flux_hist(o, hi - lo), int(o["n_accept"].sum()), hi - lo


def _worker(rank, world, port, kw, outdir):
    import torch
    import torch.distributed as dist
    from adiabatic_raytracer_amd.shard import allreduce_flux, reduce_totals
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        h, steps, n = _shard_work(rank, world, N_RAYS, kw)
        hist = torch.tensor(h, dtype=torch.float64)
        allreduce_flux(hist, world)
        tot_steps, tmax, tot_rays = reduce_totals(steps, 0.5 + rank, n, world)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), hist=hist.numpy(), steps=tot_steps, tmax=tmax,
                 rays=tot_rays)
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    from adiabatic_raytracer_amd.shard import shard_range
    for n in (0, 1, 7, 10_000_000):
        for w in (1, 2, 3, 8):
            r = [shard_range(n, i, w) for i in range(w)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(r[i][1] == r[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in r]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def test_gloo_world2_matches_single_process(tmp_path):
    import torch.multiprocessing as mp
    kw = CONFIGS["flat"]
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, kw, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    h_full, steps_full, _ = _shard_work(0, 1, N_RAYS, kw)
    for r in range(2):
        z = np.load(tmp_path / f"r{r}.npz")
        assert np.array_equal(z["hist"], h_full)  # identical batch, exact integer-valued sums
        assert int(z["steps"]) == steps_full
        assert int(z["rays"]) == N_RAYS
        assert float(z["tmax"]) == 1.5  # max over ranks
    assert h_full.sum() > 0
