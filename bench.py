#!/usr/bin/env python3
"""bench.py -- ray-steps/s (FP64) of the MI355X engine on BASELINE.json's workload.

A "step" = one pass of the hot path over one batch: RT.propagate of every segment of the
batch (RayTracer.jl:171-452: Vern6 + resonance scan + crossing polish + conversion
probability at the crossing), the binned flux of the escaping photons (plot/flux.py:38-48)
and, for N > 1, its RCCL all-reduce. Inputs are forward-tree roots sampled ON THE GPU with
the restated find_samples_new (seed 1769, Philox keyed by global ray id) BEFORE the timed
region, so they are resident in HBM when timing starts.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rays R] [--config flat|gr]

N > 1: launched by torch.distributed.run, one rank per GPU; the R rays are sharded in
contiguous blocks (strong scaling of the fixed 1e7-ray batch named by BASELINE.json).
Rank 0 prints ONE JSON line.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PEAK_FP64_TFLOPS = 78.6  # MI355X FP64 vector (= FP64 matrix) dense peak, MI355X_MICROARCH / BASELINE.md §3
PEAK_HBM_GBS = 8000.0

CONFIGS = {
    # BASELINE.json configs[1..2]: GJ dipole, flat space, m_a = 1e-5 eV, θm = 0.2, ωPul = 1, B0 = 1e14 G
    "flat": dict(theta_m=0.2, mass_a=1e-5, flat=True),
    # configs[3]: Schwarzschild GR (runner_GR_tasks.sh:10-14)
    "gr": dict(theta_m=0.0, mass_a=1e-6, flat=False),
}


def flops_per_launch(stats, fl, integrator="vern6"):
    """Algorithmic FLOPs of one launch of the integrator kernel (propagate_kernel) from its own
    counters and the instrumented per-operation counts for this configuration
    (tools/flops.json, made by tools/count_flops.cpp from the same art_core.h templates the
    kernel runs). The per-ray set-up (init_kernel) and back-transform (finalize_kernel) are
    separate kernels and are not counted here."""
    att, root, scan, interp = stats["attempts"], stats["root_steps"], stats["scan_evals"], stats["interp_evals"]
    step = fl["rk4_attempt"] if integrator == "rk4" else fl["vern6_attempt"]
    return (att * step + root * (step + fl["condition"])
            + scan * (fl["hermite_point"] + fl["condition_scan_point"])
            + interp * (fl["hermite_point"] + fl["condition"])
            + stats["accepted"] * fl["scan_certificate"])  # tried on every accepted step


# Algorithmic HBM bytes of one launch of the integrator kernel. Per segment:
# it reads erg, ln_t0 (f64), species (i8) and the 16-double fresh state init_kernel wrote
# (u0, f0, dt, c0) = 145 B, and writes the end state x_end, k_end (2 x 3 f64), u7, tau (f64)
# and status, n_accept, n_reject, n_cross (i32) = 80 B. Per recorded crossing it writes
# position, k (2 x 3 f64), t, dw (f64) = 64 B.
BYTES_PER_SEGMENT = 145 + 80
BYTES_PER_CROSSING = 64


def cpu_baseline(params, x0, k0, erg, seed, threads):
    """The oracle (oracle/art_oracle.cpp, OpenMP over rays) on a bounded sample of the same
    workload: the first rays of the same Philox-sampled forward-root batch, timed on this
    box's host cores."""
    import oracle as O
    O.build()
    po = O.make_params(**params)
    n = erg.size
    t0 = time.perf_counter()
    r = O.propagate(po, x0, k0, erg, -1.0, -30.0, 1, max_crossings=-1, nthreads=threads)
    dt = time.perf_counter() - t0
    steps = int(r["n_accept"].sum())
    return {"value": steps / dt, "unit": "ray-steps/s", "cores": threads, "kind": "port",
            "sample": f"first {n} forward-root photon segments of the seed-{seed} batch, {steps} accepted Vern6 "
                      f"steps in {dt:.1f} s on {threads} thread(s); oracle restatement (C++/OpenMP, dual-number "
                      f"gradients like ForwardDiff)"}


def host_cores():
    """CPUs this job may use: the cgroup CPU quota (cpu.max) when one is set, else the
    affinity mask. (The GPU box: 16 of a 2 x 64-core EPYC 9575F.)"""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def pcie_inclusive(eng, inp, n, accepted_per_launch, reps=2):
    """The host-buffer rate: art_propagate_host on pageable host
    arrays -- H2D of the inputs, the kernels, D2H of every output -- as a Julia ccall would
    run it. Outputs are allocated and faulted in once, outside the timing."""
    import ctypes as C
    from adiabatic_raytracer_amd._lib import CrossingBuf, SegmentOut, check, load
    lib = load()
    h = {k: inp[k].cpu().numpy() for k in ("x0", "k0", "erg", "dw", "ln_t0", "species")}
    out = {"x_end": np.ones(3 * n), "k_end": np.ones(3 * n), "u7_end": np.ones(n), "tau_end": np.ones(n),
           "status": np.ones(n, np.int32), "n_accept": np.ones(n, np.int32), "n_reject": np.ones(n, np.int32),
           "n_cross": np.ones(n, np.int32), "xc_pos": np.ones(3 * n), "xc_k": np.ones(3 * n), "xc_t": np.ones(n),
           "xc_dw": np.ones(n), "xc_p": np.ones(n)}
    P = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    so = SegmentOut(*[P(out[k]) for k in ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept", "n_reject")])
    xb = CrossingBuf(1, *[P(out[k]) for k in ("n_cross", "xc_pos", "xc_k", "xc_t", "xc_dw", "xc_p")])
    cp = eng.cp

    def run():
        check(lib.art_propagate_host(C.byref(cp), n, *[P(h[k]) for k in ("x0", "k0", "erg", "dw", "ln_t0", "species")],
                                     -1, C.byref(so), C.byref(xb)))
    run()  # staging buffers
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    dt = (time.perf_counter() - t0) / reps
    in_b = sum(a.nbytes for a in h.values())
    out_b = sum(a.nbytes for a in out.values())
    return {"value": accepted_per_launch / dt, "unit": "ray-steps/s", "ms_per_step": dt * 1e3,
            "h2d_bytes": in_b, "d2h_bytes": out_b,
            "note": "art_propagate_host on pageable host buffers (H2D + init/integrator/finalize kernels + "
                    "D2H), rank 0, same batch; value above is device-resident"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rays", type=int, default=10_000_000)
    ap.add_argument("--config", default="flat", choices=sorted(CONFIGS))
    ap.add_argument("--integrator", default="vern6", choices=["vern6", "rk4"])
    ap.add_argument("--seed", type=int, default=1769)
    ap.add_argument("--nbins", type=int, default=50)
    ap.add_argument("--streams", type=int, default=0,
                    help="batches in flight (HIP streams); 0: 1 for per-GPU batches of >= 8e6 rays, else 4 "
                         "(16 for the GR configs)")
    ap.add_argument("--cpu-rays", type=int, default=int(os.environ.get("ART_CPU_RAYS", "500000")))
    ap.add_argument("--cpu-rays-1t", type=int, default=int(os.environ.get("ART_CPU_RAYS_1T", "24000")))
    ap.add_argument("--donate", type=int, default=-1,
                    help="tail donation lanes (art_set_tail_donation); -1: auto by streams in flight")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true")
    args = ap.parse_args()
    n_shard = args.rays // max(1, int(os.environ.get("WORLD_SIZE", "1")))  # this rank's share (to within one ray)
    if args.streams <= 0:
        # the drain tail (~3 ms: the last long rays) is ~3% of a 1e7-ray pass but ~20% of the
        # 1.25e6 rays per GPU of the 8-GPU split; overlapping passes (with tail donation, below)
        # hides most of it there. Measured per shard size with donation
        # (profiles/r02d_streams_by_shard_donation.txt): 1e6-5e6 rays best with 3 passes in
        # flight; round 3 (tail kernel, two-level donation): 1.25e6 rays 3.16e9 on 3 streams,
        # 3.31e9 on 4, 3.30e9 on 6, so 4. The GR batch is bound by its longest ray (~185 ms
        # alone on the tail kernel), so only more passes in flight amortise it: 4.2e8 on 3,
        # 6.3e8 on 6, 5.9-6.2e8 on 8, 7.4-8.7e8 on 12, 7.8-9.8e8 on 16 across fresh boxes
        # (profiles/r03grv_gr_streams_variance.txt), so 16 for the GR configs. Overlapped launches stretch each other's measured duration, so
        # the single-GPU headline (1e7 rays) runs one pass at a time and its roofline is the
        # kernel's own (2 passes with donation: +1%).
        gr = not CONFIGS[args.config].get("flat", False)
        args.streams = 1 if n_shard >= 8_000_000 else (16 if gr else 4)
    # concurrent passes need a hardware queue each (read at HIP init; the image's default is 4)
    if args.streams > 3 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < args.streams + 1:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(16, args.streams + 1))

    import torch
    import torch.distributed as dist

    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    from adiabatic_raytracer_amd.shard import allreduce_flux, reduce_totals, shard_range

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N > 1 path on a one-GPU box: every rank on one device, gloo
    # (ART_BENCH_DEVICE / ART_BENCH_BACKEND); the real runs use one GPU per rank and RCCL
    if "ART_BENCH_DEVICE" in os.environ:
        local = int(os.environ["ART_BENCH_DEVICE"])
    backend = os.environ.get("ART_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    params = A.Params(integrator=args.integrator, **CONFIGS[args.config])
    eng = Engine(params, device=local)
    # contiguous shard of the global batch; Philox keyed by global ray id -> GPU-count independent
    lo, hi = shard_range(args.rays, rank, world)
    n = hi - lo
    t_s = time.perf_counter()
    inp = eng.forward_roots(n, seed=args.seed, ray_offset=lo)
    torch.cuda.synchronize()
    sample_s = time.perf_counter() - t_s
    # `streams` batches in flight: step i runs on stream i % streams with its own outputs, so
    # the drain tail of one pass (its last long rays on a few CUs) overlaps the next pass's
    # bulk instead of idling the GPU. Each launch has its own scratch (include/art.h).
    if args.donate < 0:
        # tail donation only pays when another pass in flight can take the freed CU slots:
        # 1e6 rays on 3 streams +9%, 1.25e6 +6%; a lone pass loses 0.6-1.7% (its donated rays
        # resume only after the pass; profiles/r02d_tail_donation.txt)
        args.donate = 16 if args.streams > 1 else 0
    eng.set_tail_donation(args.donate)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(args.streams - 1)]
    outs = [eng.alloc_out(n, capacity=1) for _ in streams]
    hists = [torch.zeros(2 * args.nbins, dtype=torch.float64, device=eng.device) for _ in streams]
    for st_ in streams[1:]:
        st_.wait_stream(streams[0])  # the sampled inputs and the outputs' initialisation
    out, hist = outs[0], hists[0]

    def one_step(i):
        k = i % len(streams)
        with torch.cuda.stream(streams[k]):
            eng.propagate(inp, outs[k], max_crossings=-1)
            hists[k].zero_()
            eng.flux_histogram(outs[k], inp["species"], None, args.nbins, hists[k])
            allreduce_flux(hists[k], world)  # the only data-path collective: the binned flux (RCCL over xGMI)

    for i in range(args.warmup):
        one_step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        one_step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # per-launch integrator durations (HIP events on each launch's own stream) and the
    # launch's counters; every step integrates the same batch, so its accepted steps are
    # the same each time (checked against the outputs)
    kms_buf = (C.c_double * args.steps)()
    got = A._lib.load().art_recent_kernel_ms(args.steps, kms_buf)
    kernel_ms = list(kms_buf)[:max(0, got)]
    eng.kernel_ms()  # latches the last launch's counters
    stats_last = A.raytracer.last_stats()
    k_last = (args.warmup + args.steps - 1) % len(streams)
    out, hist = outs[k_last], hists[k_last]
    assert int(out["n_accept"].sum().item()) == stats_last["accepted"]
    accepted = stats_last["accepted"] * args.steps
    # whole-job aggregates: Σ ray-steps over ranks / max wall time over ranks
    total_steps, t_max, total_rays = reduce_totals(accepted, elapsed, n, world, device=eng.device)

    if rank == 0:
        fl_all = json.load(open(os.path.join(HERE, "tools", "flops.json")))
        fl, fl_r1 = fl_all[args.config], fl_all[args.config + "_round1"]
        kms = float(np.mean(kernel_ms))
        fpl = flops_per_launch(stats_last, fl, args.integrator)
        # with several passes in flight the launches overlap, so one launch's own duration
        # covers the device only in part: the rate is then priced on the wall per launch
        # (the overlapped launches back to back), and kernel_ms stays each launch's duration
        basis_ms = kms if len(streams) == 1 else elapsed * 1e3 / args.steps
        achieved = fpl / (basis_ms * 1e-3) / 1e12
        st = out["status"].cpu().numpy()
        traffic, traffic_src = None, None
        pmc_path = os.path.join(HERE, "profiles", "pmc_summary.json")
        if os.path.exists(pmc_path):
            pm = json.load(open(pmc_path))
            # only a PMC pass of this very library build and workload counts
            import hashlib
            sha = hashlib.sha256(open(A._lib.load()._name, "rb").read()).hexdigest()
            if pm.get("workload") == f"{args.config}:{n}" and pm.get("libart_sha256") == sha:
                traffic = pm.get("hbm_bytes_per_launch")
                traffic_src = ("stored PMC pass of this libart.so build (profiles/pmc_summary.json, sha "
                               f"{sha[:12]}, tools/pmc_passes.sh: FETCH_SIZE/WRITE_SIZE in separate passes, "
                               "calibrated by tools/calib_hbm.hip); not measured in this run")
        ncross = int((out["n_cross"].clamp(max=out["capacity"])).sum().item())
        att = (out["n_accept"] + out["n_reject"]).double()
        q = torch.quantile(att[:min(n, 1 << 24)], torch.tensor([0.5, 0.99, 0.999], dtype=torch.float64,
                                                               device=att.device)).tolist()
        attempt_dist = {"mean": float(att.mean()), "p50": q[0], "p99": q[1], "p999": q[2], "max": float(att.max())}
        alg_bytes = n * BYTES_PER_SEGMENT + ncross * BYTES_PER_CROSSING
        line = {
            "metric": "ray-steps/sec (FP64), 10^7-ray GJ-dipole batch",
            "value": total_steps / t_max,
            "unit": "ray-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: forward-tree roots sampled on the GPU by the restated find_samples_new (Philox seed 1769)",
            "config": {"workload": f"{total_rays} photon segments, GJ dipole, "
                                   f"{'flat space' if params.flat else 'Schwarzschild GR'}, {args.integrator}",
                       "baseline_config": "configs[2] (1e7 rays, sharded over the GPUs)" if args.rays == 10_000_000
                       else f"{args.rays} rays",
                       "m_a_eV": params.mass_a, "theta_m": params.theta_m, "omega_pul": params.omega_pul,
                       "B0_G": params.B0, "rNS_km": params.rNS, "abstol": params.abstol, "reltol": params.reltol,
                       "interp_points": params.interp_points, "parallelism": f"rays sharded x{world}",
                       "streams": args.streams, "tail_donation": args.donate},
            "roofline": {"bound": "fp64-valu", "achieved": achieved, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / PEAK_FP64_TFLOPS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": f"propagate_kernel<{'RK4' if args.integrator == 'rk4' else 'Vern6'}>", "kernel_ms": kms,
                         "flops_per_launch": fpl, "flops_per_ray_step": fpl / stats_last["accepted"],
                         "time_basis": "launch duration (HIP events)" if len(streams) == 1
                         else f"wall per launch ({len(streams)} overlapping passes)", "basis_ms": basis_ms,
                         "frac_round1_flop_table": flops_per_launch(stats_last, fl_r1, args.integrator) / (basis_ms * 1e-3)
                                                   / 1e12 / PEAK_FP64_TFLOPS,
                         "achieved_wall": fpl * args.steps / elapsed / 1e12,
                         "note": "FP64 VALU-bound (state in VGPRs, ~1 B of HBM per ray-step); peak = 78.6 TFLOP/s "
                                 "FP64 (vector = matrix dense peak). FLOPs from the kernel's counters x "
                                 "tools/flops.json (instrumented restatement).",
                         "hbm": {"algorithmic_bytes_per_launch": alg_bytes,
                                 "achieved_GBs": alg_bytes / (basis_ms * 1e-3) / 1e9, "peak_GBs": PEAK_HBM_GBS,
                                 "frac": alg_bytes / (basis_ms * 1e-3) / 1e9 / PEAK_HBM_GBS}},
            "kernel_stats": stats_last,
            "status_counts": np.bincount(st, minlength=5).tolist(),
            "attempts_per_ray": attempt_dist,
            "ic_sampling_s": sample_s,
        }
        if not args.no_pcie:
            line["pcie_inclusive"] = pcie_inclusive(eng, inp, n, stats_last["accepted"])
        if world == 1 and not args.no_cpu_baseline:
            threads = int(os.environ.get("ART_CPU_THREADS", str(host_cores())))

            def sample(m):
                xs = inp["x0"].view(3, n)[:, :m].cpu().numpy().reshape(-1)
                ks = inp["k0"].view(3, n)[:, :m].cpu().numpy().reshape(-1)
                return xs, ks, inp["erg"][:m].cpu().numpy()
            cfg = CONFIGS[args.config] | {"integrator": 0}
            m = min(args.cpu_rays, n)
            line["cpu_baseline"] = cpu_baseline(cfg, *sample(m), args.seed, threads)
            # and one core: the reference's own model is one single-threaded process per ray batch
            m1 = min(args.cpu_rays_1t, n)
            line["cpu_baseline"]["one_thread"] = cpu_baseline(cfg, *sample(m1), args.seed, 1)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
