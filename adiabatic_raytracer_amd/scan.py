"""The parameter scan of BASELINE.json configs[4]: 32 (m_a, B0, P_NS) grid points, each a batch
of forward-tree root segments, spread over the GPUs of one node.

The reference scans parameters by launching one Gen_Samples.jl process per grid point
(jonas_test_analyses/runner_tree.sh:1-12 sweeps MassA x Axg). Here every rank takes whole
grid points (replicas: no collective on the data path) and runs, per point, the same
pipeline as bench.py: sample conversion points on the GPU (Philox keyed by seed and ray
id), RT.propagate every segment, and bin the escaping photons (plot/flux.py:38-48). Rank 0
gathers one record per point at the end.

    python -m adiabatic_raytracer_amd.scan [--rays R] [--points K] [--out FILE]
    python -m torch.distributed.run --nproc-per-node N -m adiabatic_raytracer_amd.scan ...
"""
from __future__ import annotations

import argparse
import itertools
import json
import math
import os
import time

# m_a in {1, 2, 5, 10} x 1e-6 eV, B0 in {2.5, 5, 10, 20} x 1e13 G,
# P in {0.5, 1} s (ωPul = 2π/P); GJ dipole, θm = 0.2, flat space
MASSES = (1e-6, 2e-6, 5e-6, 1e-5)
FIELDS = (2.5e13, 5e13, 1e14, 2e14)
PERIODS = (0.5, 1.0)


def scan_grid(theta_m: float = 0.2, flat: bool = True) -> list[dict]:
    """The 32 grid points as Params keyword sets, in (m_a, B0, P) lexicographic order."""
    return [dict(mass_a=m, B0=b, omega_pul=2.0 * math.pi / per, theta_m=theta_m, flat=flat)
            for m, b, per in itertools.product(MASSES, FIELDS, PERIODS)]


def points_of_rank(n_points: int, rank: int, world: int) -> list[int]:
    """Grid points owned by `rank`: round robin, so every rank gets points of every mass."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    return list(range(rank, n_points, world))


def run_point(kw: dict, rays: int, seed: int = 1769, nbins: int = 50, device: int = 0) -> dict:
    """One grid point on one GPU: forward-tree roots -> propagate -> flux histogram."""
    import torch

    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    p = A.Params(**kw)
    eng = Engine(p, device=device)
    max_r = p.max_r()
    rec = dict(kw, rays=rays, max_r_km=max_r)
    if max_r < p.rNS:  # no conversion surface outside the star (MainRunner.jl:387-396)
        return dict(rec, skipped="maxR < rNS")
    t0 = time.perf_counter()
    inp = eng.forward_roots(rays, seed=seed)
    out = eng.propagate(inp, max_crossings=-1)
    hist = eng.flux_histogram(out, inp["species"], None, nbins)
    torch.cuda.synchronize()
    kernel_ms = eng.kernel_ms()  # synchronizes and latches the launch's counters
    st = A.raytracer.last_stats()
    status = torch.bincount(out["status"].long(), minlength=5).tolist()
    return dict(rec, seconds=time.perf_counter() - t0, kernel_ms=kernel_ms, accepted=st["accepted"],
                attempts=st["attempts"], status_counts=status, flux_photon=hist[nbins:].tolist())


def run_scan(rays: int, n_points: int | None = None, seed: int = 1769, run=run_point) -> list[dict]:
    """This rank's share of the grid; with WORLD_SIZE > 1 the records are gathered on every
    rank (all_gather_object) and returned in grid order."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    grid = scan_grid()[:n_points]
    mine = [dict(run(grid[i], rays, seed, device=local), point=i) for i in points_of_rank(len(grid), rank, world)]
    if world == 1:
        return mine
    parts = [None] * world
    dist.all_gather_object(parts, mine)
    return sorted((r for part in parts for r in part), key=lambda r: r["point"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=1_000_000)
    ap.add_argument("--points", type=int, default=None)
    ap.add_argument("--seed", type=int, default=1769)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    recs = run_scan(args.rays, args.points, args.seed)
    if int(os.environ.get("RANK", "0")) == 0:
        lines = "\n".join(json.dumps(r) for r in recs)
        if args.out:
            with open(args.out, "w") as fh:
                fh.write(lines + "\n")
        print(lines, flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
