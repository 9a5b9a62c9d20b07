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


def run_points(kws: list[dict], rays: int, seed: int = 1769, nbins: int = 50, device: int = 0,
               streams: int = 8, donate: int = 0) -> tuple[list[dict], dict]:
    """Several grid points on one GPU, `streams` of them in flight. Every point's forward
    roots are sampled first; then the points are propagated on `streams` HIP streams, longest
    expected drain (largest conversion radius) first, each next point on the first stream to
    go idle (dispatch). Each launch has its own device scratch (include/art.h), so a point's
    drain tail (its last long rays on a few CUs; 20-840 ms per 1e6-ray point) overlaps the
    other points' bulk, and each point's flux is binned on its stream. Streams run
    concurrently only up to the process's hardware queues: main() raises GPU_MAX_HW_QUEUES
    to the stream count (HIP's default is 4; 8 streams measured fastest on one MI355X, 16
    slower). Returns the per-point records (grid order) and a summary of the propagate
    phase (wall time, Σ accepted steps)."""
    import ctypes as C

    import torch

    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    main = torch.cuda.current_stream()
    ss = [main] + [torch.cuda.Stream() for _ in range(max(1, streams) - 1)]
    for s_ in ss[1:]:
        s_.wait_stream(main)
    t0 = time.perf_counter()
    engs, recs = [], []
    try:
        for kw in kws:
            p = A.Params(**kw)
            rec = dict(kw, rays=rays, max_r_km=p.max_r())
            recs.append(rec)
            if rec["max_r_km"] < p.rNS:  # no conversion surface outside the star (MainRunner.jl:387-396)
                rec["skipped"] = "maxR < rNS"
                engs.append(None)
            else:
                engs.append(Engine(p, device=device))
                engs[-1].set_tail_donation(donate)
                engs[-1].set_graduation(0 if len(ss) > 1 else -1)  # (passes in flight: off)
                # samplers in flight: the 3-wave build for every line (per device; 0.503-0.508 -> 0.484 s
                # of sampling, profiles/r05ah_scan_sampler_waves.txt)
                engs[-1].set_sampler_waves(3 if len(ss) > 1 else 0)
        # Longest expected drain first: a point's kernel time grows with its conversion radius
        # (maxR: 29 km -> 20 ms ... 342 km -> 835 ms per 1e6 rays, profiles/r02b_scan_order.txt),
        # and the longest single ray bounds the whole scan, so it should start at once.
        live = sorted((i for i, e in enumerate(engs) if e is not None), key=lambda i: -recs[i]["max_r_km"])
        inps, outs, hists = {}, {}, {}

        def sample(i):  # the samplers' tails overlap too
            inps[i] = engs[i].forward_roots(rays, seed=seed)

        dispatch(live, sample, ss)
        torch.cuda.synchronize()
        t_sample = time.perf_counter() - t0

        def prop(i):
            outs[i] = engs[i].propagate(inps[i], max_crossings=-1)
            hists[i] = engs[i].flux_histogram(outs[i], inps[i]["species"], None, nbins)

        t1 = time.perf_counter()
        order = dispatch(live, prop, ss)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t1
    finally:
        # the device's defaults again (graduation, sampler build) for every device configured,
        # also when a point's dispatch raised: they are per-device settings later Engines inherit
        for e in engs:
            if e is not None:
                e.set_graduation(-1)
                e.set_sampler_waves(0)
    k = len(order)
    ms = (C.c_double * max(1, k))()
    got = A._lib.load().art_recent_kernel_ms(k, ms)
    # the ring holds the device's last min(k, 64) propagate launches, oldest first: they are the
    # last `got` points of the dispatch order only when all k were recorded (got == k); past the
    # ring's 64 entries the durations are not attributed at all rather than to the wrong points
    kms = dict(zip(order[-got:], list(ms)[:got])) if got == k else {}
    acc_total = 0
    for i in live:
        o = outs[i]
        acc = int(o["n_accept"].sum().item())
        att = acc + int(o["n_reject"].sum().item())
        acc_total += acc
        recs[i].update(kernel_ms=kms.get(i), accepted=acc, attempts=att,
                       status_counts=torch.bincount(o["status"].long(), minlength=5).tolist(),
                       flux_photon=hists[i][nbins:].tolist())
    summary = {"points": k, "streams": len(ss), "order": order, "sample_s": t_sample, "propagate_wall_s": wall,
               "accepted": acc_total, "kernel_ray_steps_per_s": acc_total / wall if wall > 0 else None}
    return recs, summary


def dispatch(items, launch, streams, poll_s=2e-4):
    """Runs launch(item) on the first of `streams` that has gone idle, in item order: one
    item per stream up front, then each next item on whichever stream finishes first (an
    event per launch, polled from the host). A round-robin assignment would queue item
    k + len(streams) behind item k even when item k holds a long drain tail (a 1e6-ray
    scan point's last ray can take ~0.8 s on its own) while the other streams sit idle.
    Returns the items in launch order."""
    import torch
    order, busy = [], {}
    todo = list(items)
    free = list(range(len(streams)))
    while todo or busy:
        while todo and free:
            j = free.pop(0)
            it = todo.pop(0)
            with torch.cuda.stream(streams[j]):
                launch(it)
                ev = torch.cuda.Event()
                ev.record()
            busy[j] = ev
            order.append(it)
        if not todo:
            break
        done = [j for j, ev in busy.items() if ev.query()]
        if not done:
            time.sleep(poll_s)
        for j in done:
            del busy[j]
            free.append(j)
    return order


def run_scan(rays: int, n_points: int | None = None, seed: int = 1769, run=None, streams: int = 8, donate: int = 0):
    """This rank's share of the grid (run_points, or `run` point by point); with
    WORLD_SIZE > 1 the records are gathered on every rank (all_gather_object) and returned in
    grid order."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    grid = scan_grid()[:n_points]
    idx = points_of_rank(len(grid), rank, world)
    if run is None:
        recs, _ = run_points([grid[i] for i in idx], rays, seed, device=local, streams=streams, donate=donate)
        mine = [dict(r, point=i) for r, i in zip(recs, idx)]
    else:
        mine = [dict(run(grid[i], rays, seed, device=local), point=i) for i in idx]
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
    ap.add_argument("--streams", type=int, default=8)
    ap.add_argument("--donate", type=int, default=16,
                    help="tail donation lanes (art_set_tail_donation): the drained tails resume packed, then one "
                         "wave per ray (tail kernel)")
    args = ap.parse_args()
    # concurrent kernels need hardware queues: one per stream in flight (read at HIP init)
    want = min(16, max(4, args.streams))
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < want:
        os.environ["GPU_MAX_HW_QUEUES"] = str(want)
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    recs = run_scan(args.rays, args.points, args.seed, streams=args.streams, donate=args.donate)
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
