#!/usr/bin/env python3
"""bench.py -- ray-steps/s (FP64) of the MI355X engine on BASELINE.json's workload.

A "step" = one pass of the hot path over one batch: RT.propagate of every segment of the
batch (RayTracer.jl:171-452: Vern6 + resonance scan + crossing polish + conversion
probability at the crossing), the binned flux of the escaping photons (plot/flux.py:38-48)
and, for N > 1, its RCCL all-reduce. Inputs are forward-tree roots sampled on the GPU with
the restated find_samples_new (seed 1769, Philox keyed by global ray id) BEFORE the timed
region (reported apart, `ic_sampling_s`) and copied to host arrays.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rays R] [--config flat|gr]

The timed region is BASELINE.md §2 / SURVEY §8(d)'s: H2D + kernels + D2H. Each step hands
the batch to art_propagate_host_flux as pageable host arrays (what a Julia ccall from
MainRunner.jl:179-190 passes) and gets every output back in host arrays, so `value` is the
drop-in rate. The same passes on device-resident inputs are reported as side figures
(`device_resident`, and `device_resident_in_flight` with several batches on as many streams).

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


def cpu_baseline(params, x0, k0, erg, seed, threads, same_algorithm=True):
    """A CPU figure on a bounded sample of the same workload (the first rays of the same
    Philox-sampled forward-root batch), timed on this box's host cores.
    same_algorithm: the engine's algorithm on the host (tools/cpu_same.cpp: art_core.h's
    physics compiled for the CPU, scalar Vern6 + certified 50-point scan, OpenMP over rays);
    else the oracle (oracle/art_oracle.cpp), whose dual-number gradients cost what the
    reference's ForwardDiff passes do."""
    import oracle as O
    O.build()
    po = O.make_params(**params)
    n = erg.size
    if same_algorithm:
        sys.path.insert(0, os.path.join(HERE, "tools"))
        import cpu_same
        cpu_same.build()
        t0 = time.perf_counter()
        r = cpu_same.propagate(po, x0, k0, erg, -1.0, -30.0, 1, max_crossings=-1, nthreads=threads)
        what = ("the engine's algorithm on the host (tools/cpu_same.cpp: art_core.h compiled for the CPU, scalar "
                "Vern6 + certified 50-point scan + re-step polish, OpenMP over rays)")
    else:
        t0 = time.perf_counter()
        r = O.propagate(po, x0, k0, erg, -1.0, -30.0, 1, max_crossings=-1, nthreads=threads)
        what = "oracle restatement (C++/OpenMP, dual-number gradients like the reference's ForwardDiff)"
    dt = time.perf_counter() - t0
    steps = int(r["n_accept"].sum())
    return {"value": steps / dt, "unit": "ray-steps/s", "cores": threads, "kind": "port",
            "variant": "same-algorithm" if same_algorithm else "forwarddiff-restatement",
            "sample": f"first {n} forward-root photon segments of the seed-{seed} batch, {steps} accepted Vern6 "
                      f"steps in {dt:.1f} s on {threads} thread(s); {what}"}


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


def bind_to_gpu_node(device):
    """Binds this rank (its main thread, and every thread it starts later: libart's copy pool,
    gatherers, lane workers) to the CPUs of the NUMA node its GPU hangs off, so the pageable host
    arrays and the pinned staging are first touched there; the host path measured up to 3.9 ms
    slower per 1e7-ray call from the far node (profiles/r05r_numa_binding.txt). Returns the node,
    or None when sysfs does not tell (nothing is changed then). ART_BENCH_NO_NUMA=1: no binding."""
    if os.environ.get("ART_BENCH_NO_NUMA"):
        return None
    import glob
    import torch
    try:
        bus = int(torch.cuda.get_device_properties(device).pci_bus_id)
        for d in glob.glob("/sys/bus/pci/devices/*"):
            parts = os.path.basename(d).split(":")
            if len(parts) != 3 or int(parts[1], 16) != bus:
                continue
            cls = open(os.path.join(d, "class")).read().strip()
            if not (cls.startswith("0x03") or cls.startswith("0x12")):  # display / processing accelerator
                continue
            node = int(open(os.path.join(d, "numa_node")).read().strip())
            if node < 0:
                return None
            cpus = set()
            for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
                lo, _, hi = part.partition("-")
                cpus.update(range(int(lo), int(hi or lo) + 1))
            cpus &= os.sched_getaffinity(0)
            if not cpus:
                return None
            os.sched_setaffinity(0, cpus)
            return node
    except (OSError, ValueError, AttributeError):
        return None
    return None


def host_arrays(inp, n):
    """This rank's batch as a Julia caller holds it (MainRunner.jl:179-190 hands host arrays
    to propagate): pageable numpy inputs, and output arrays allocated and faulted in once."""
    h = {k: np.ascontiguousarray(inp[k].cpu().numpy()) for k in ("x0", "k0", "erg", "dw", "ln_t0", "species")}
    out = {"x_end": np.ones(3 * n), "k_end": np.ones(3 * n), "u7_end": np.ones(n), "tau_end": np.ones(n),
           "status": np.ones(n, np.int32), "n_accept": np.ones(n, np.int32), "n_reject": np.ones(n, np.int32),
           "n_cross": np.ones(n, np.int32), "xc_pos": np.ones(3 * n), "xc_k": np.ones(3 * n), "xc_t": np.ones(n),
           "xc_dw": np.ones(n), "xc_p": np.ones(n)}
    return h, out


def timed(run, steps, warmup, world, sync, drain=lambda: None):
    """W untimed warmup steps, then EXACTLY `steps` steps bracketed by a barrier and a device
    synchronize on both sides; returns this rank's elapsed seconds. `drain` completes the steps
    still in flight (host calls submitted asynchronously) before each synchronize."""
    import torch.distributed as dist
    for i in range(warmup):
        run(i)
    drain()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        run(warmup + i)
    drain()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    return time.perf_counter() - t0


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
                    help="device-resident side figure: batches in flight (HIP streams); 0: 1 for per-GPU batches "
                         "of >= 8e6 rays, else 4 (16 for the GR configs)")
    # CPU samples (about 5-15 s each on the GPU box's 16 cores): the same-algorithm port on all
    # cores and on one, then the dual-number oracle on all cores and on one
    ap.add_argument("--cpu-rays", type=int, default=int(os.environ.get("ART_CPU_RAYS", "3000000")))
    ap.add_argument("--cpu-rays-1t", type=int, default=int(os.environ.get("ART_CPU_RAYS_1T", "300000")))
    ap.add_argument("--cpu-rays-oracle", type=int, default=int(os.environ.get("ART_CPU_RAYS_ORACLE", "250000")))
    ap.add_argument("--cpu-rays-oracle-1t", type=int, default=int(os.environ.get("ART_CPU_RAYS_ORACLE_1T", "12000")))
    ap.add_argument("--donate", type=int, default=-1,
                    help="tail donation lanes for the device-resident passes in flight; -1: auto")
    ap.add_argument("--inflight", type=int, default=0,
                    help="host calls in flight per rank (art_propagate_host_flux_async: the next batch's uploads and "
                         "first rays overlap this one's drain); 0: 1 for per-GPU batches of >= 8e6 rays, else 2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-device", action="store_true", help="skip the device-resident side figures")
    ap.add_argument("--no-pcie", action="store_true", help="(compat) same as --no-device")
    args = ap.parse_args()
    n_shard = args.rays // max(1, int(os.environ.get("WORLD_SIZE", "1")))  # this rank's share (to within one ray)
    gr = not CONFIGS[args.config].get("flat", False)
    if args.inflight <= 0:
        args.inflight = 1 if n_shard >= 8_000_000 else 2
    if args.streams <= 0:
        # device-resident side figure only (value is one host call per batch). The drain tail
        # (~3 ms: the last long rays) is ~3% of a 1e7-ray pass but ~20% of the 1.25e6 rays per GPU
        # of the 8-GPU split; overlapping passes (with tail donation) hides most of it: 1.25e6
        # rays 3.31e9 on 4 streams. The GR batch is bound by its longest ray (~185 ms alone on the
        # tail kernel), so only more passes in flight amortise it (profiles/r03grv_gr_streams_
        # variance.txt): 16 for the GR configs.
        args.streams = 1 if n_shard >= 8_000_000 else (16 if gr else 4)
    # concurrent passes need a hardware queue each (read at HIP init; the image's default is 4)
    if args.streams > 3 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < args.streams + 1:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(16, args.streams + 1))

    import torch
    import torch.distributed as dist

    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    from adiabatic_raytracer_amd._lib import CrossingBuf, SegmentOut, check
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
    numa_node = bind_to_gpu_node(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    params = A.Params(integrator=args.integrator, **CONFIGS[args.config])
    eng = Engine(params, device=local)
    lib = A._lib.load()
    # contiguous shard of the global batch; Philox keyed by global ray id -> GPU-count independent
    lo, hi = shard_range(args.rays, rank, world)
    n = hi - lo
    t_s = time.perf_counter()
    inp = eng.forward_roots(n, seed=args.seed, ray_offset=lo)
    torch.cuda.synchronize()
    sample_s = time.perf_counter() - t_s
    hist_dev = world > 1 and backend == "nccl"  # RCCL reduces device tensors, gloo host ones

    def sync():
        torch.cuda.synchronize()

    # ---- the headline: BASELINE §2 / SURVEY §8(d)'s timed region, H2D + kernels + D2H ----
    # One step = art_propagate_host_flux on this rank's pageable batch (inputs up, the init /
    # integrator / finalize kernels, every output back into the caller's arrays, the batch's
    # binned flux from the outputs while they are in HBM) and the all-reduce of that flux over
    # the ranks (RCCL over xGMI; the path's only exchange, north_star).
    h, out0 = host_arrays(inp, n)
    P = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    # one set of output arrays per call in flight (the inputs are only read)
    sets = []
    for j in range(args.inflight):
        o = host_arrays(inp, n)[1] if j else out0
        sets.append({"out": o, "flux": np.zeros(2 * args.nbins),
                     "so": SegmentOut(*[P(o[k]) for k in ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept",
                                                         "n_reject")]),
                     "xb": CrossingBuf(1, *[P(o[k]) for k in ("n_cross", "xc_pos", "xc_k", "xc_t", "xc_dw", "xc_p")])})
    flux_red = {}
    pending = []  # (ticket, set) of the calls in flight, oldest first
    ins = [P(h[k]) for k in ("x0", "k0", "erg", "dw", "ln_t0", "species")]

    def reduce_flux(st):
        t = torch.from_numpy(st["flux"].copy())
        flux_red["host"] = allreduce_flux(t.to(eng.device) if hist_dev else t, world)
        flux_red["set"] = st

    def wait_oldest():
        tk, st = pending.pop(0)
        check(lib.art_host_wait(tk))
        reduce_flux(st)

    def host_step(i):
        st = sets[i % args.inflight]
        if args.inflight == 1:
            check(lib.art_propagate_host_flux(C.byref(eng.cp), n, *ins, -1, C.byref(st["so"]), C.byref(st["xb"]),
                                              args.nbins, P(st["flux"])))
            reduce_flux(st)
            return
        if len(pending) == args.inflight:
            wait_oldest()
        tk = C.c_int64(-1)
        check(lib.art_propagate_host_flux_async(C.byref(eng.cp), n, *ins, -1, C.byref(st["so"]), C.byref(st["xb"]),
                                                args.nbins, P(st["flux"]), C.byref(tk)))
        pending.append((tk.value, st))

    def drain():
        while pending:
            wait_oldest()

    A.raytracer.host_path_counters(reset=True)
    for i in range(args.warmup):  # (the first call also allocates the pinned staging and streams)
        host_step(i)
    drain()
    cnt_w = A.raytracer.host_path_counters(reset=True)
    host_s = timed(host_step, args.steps, 0, world, sync, drain)
    hout = flux_red["set"]["out"]  # (the last call's outputs)
    cnt = A.raytracer.host_path_counters()
    # every timed pass ran the path its size selects, and none gave up and ran twice
    assert cnt["stream_giveups"] == 0, f"streamed host pipeline gave up inside the timed passes: {cnt}"
    assert cnt["calls"] == args.steps, cnt
    kms_buf = (C.c_double * args.steps)()
    got = lib.art_recent_kernel_ms(args.steps, kms_buf)
    host_kms = list(kms_buf)[:max(0, got)]
    host_span = A.raytracer.recent_kernel_span_ms(args.steps)  # the same launches, in-kernel clock stamps
    host_stats = A.raytracer.last_stats()
    assert int(hout["n_accept"].sum()) == host_stats["accepted"]
    host_steps_total, host_t_max, total_rays = reduce_totals(host_stats["accepted"] * args.steps, host_s, n, world,
                                                             device=eng.device if hist_dev else None)
    host_status = hout["status"].copy()

    # ---- side figure: the same passes on device-resident inputs (art_propagate_device) ----
    dev = None
    if not (args.no_device or args.no_pcie):
        donate = args.donate if args.donate >= 0 else (16 if args.streams > 1 else 0)

        def device_run(nstreams, donate_lanes, steps, warmup):
            eng.set_tail_donation(donate_lanes)
            eng.set_graduation(0 if nstreams > 1 else -1)  # (batches in flight: off, include/art.h)
            # (non-blocking streams, as a host keeping batches in flight uses: the GR batch's
            # early graduation runs only on one, include/art.h)
            streams = [torch.cuda.Stream() for _ in range(nstreams)]
            outs = [eng.alloc_out(n, capacity=1) for _ in streams]
            hists = [torch.zeros(2 * args.nbins, dtype=torch.float64, device=eng.device) for _ in streams]
            for st_ in streams:
                st_.wait_stream(torch.cuda.current_stream())  # the sampled inputs and the outputs' initialisation

            def one_step(i):
                k = i % len(streams)
                with torch.cuda.stream(streams[k]):
                    eng.propagate(inp, outs[k], max_crossings=-1)
                    hists[k].zero_()
                    eng.flux_histogram(outs[k], inp["species"], None, args.nbins, hists[k])
                    allreduce_flux(hists[k], world)
            el = timed(one_step, steps, warmup, world, sync)
            kb = (C.c_double * steps)()
            g = lib.art_recent_kernel_ms(steps, kb)
            span = A.raytracer.recent_kernel_span_ms(steps)
            eng.kernel_ms()  # latches the last launch's counters
            st = A.raytracer.last_stats()
            k_last = (warmup + steps - 1) % len(streams)
            assert int(outs[k_last]["n_accept"].sum().item()) == st["accepted"]
            tot, tmax, _ = reduce_totals(st["accepted"] * steps, el, n, world, device=eng.device)
            eng.set_tail_donation(-1)
            eng.set_graduation(-1)
            return {"value": tot / tmax, "ms_per_step": tmax / steps * 1e3, "kernel_ms": float(np.mean(list(kb)[:g])),
                    "kernel_span_ms": float(np.mean(span)) if span else None,
                    "streams": nstreams, "tail_donation": donate_lanes, "elapsed_s": el, "stats": st,
                    "hist": hists[k_last].cpu().numpy()}
        dev = {"one": device_run(1, -1, args.steps, args.warmup)}  # (-1: the library default by geometry)
        if args.streams > 1:
            dev["many"] = device_run(args.streams, donate, args.steps * max(1, min(args.streams, 4)), args.warmup)

    if rank == 0:
        fl_all = json.load(open(os.path.join(HERE, "tools", "flops.json")))
        fl, fl_r1 = fl_all[args.config], fl_all[args.config + "_round1"]
        import hashlib
        sha = hashlib.sha256(open(lib._name, "rb").read()).hexdigest()
        pm = {}
        pmc_path = os.path.join(HERE, "profiles", "pmc_summary.json")
        if os.path.exists(pmc_path):
            pm = json.load(open(pmc_path))
            # only a PMC pass of this very library build and workload counts
            if not (pm.get("workload") == f"{args.config}:{n}" and pm.get("libart_sha256") == sha):
                pm = {}

        def traffic(kind):
            k = pm.get("kernels", {}).get(kind)
            return (k["hbm_bytes_per_launch"], ("stored PMC pass of this libart.so build (profiles/pmc_summary.json, "
                                                f"sha {sha[:12]}, kernel {k['kernel']}, tools/pmc_passes.sh: FETCH_SIZE/"
                                                "WRITE_SIZE in separate passes, calibrated by tools/calib_hbm.hip); not "
                                                "measured in this run")) if k else (None, None)

        kms = float(np.mean(host_kms))
        fpl = flops_per_launch(host_stats, fl, args.integrator)
        host_ms = host_t_max / args.steps * 1e3
        # one call at a time: the integrator launch's own duration; calls in flight overlap each
        # other's launches, so the wall per call is the basis (as for device_resident_in_flight)
        basis_ms = kms if args.inflight == 1 else host_ms
        ncross = int(np.minimum(hout["n_cross"], 1).sum())
        att = (hout["n_accept"].astype(np.float64) + hout["n_reject"])
        q = np.quantile(att, [0.5, 0.99, 0.999])
        attempt_dist = {"mean": float(att.mean()), "p50": q[0], "p99": q[1], "p999": q[2], "max": float(att.max())}
        alg_bytes = n * BYTES_PER_SEGMENT + ncross * BYTES_PER_CROSSING
        streamed = cnt["streamed"] == args.steps
        kname = (f"propagate_kernel<{'RK4' if args.integrator == 'rk4' else 'Vern6'}"
                 f"{', streamed (DON=3)' if streamed else ''}>")
        tr, tr_src = traffic("streamed" if streamed else "device")
        in_b = sum(a.nbytes for a in h.values())
        out_b = sum(a.nbytes for a in hout.values())
        line = {
            "metric": "ray-steps/sec (FP64), 10^7-ray GJ-dipole batch",
            "value": host_steps_total / host_t_max,
            "unit": "ray-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": host_ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: forward-tree roots sampled on the GPU by the restated find_samples_new (Philox seed "
                    f"{args.seed}), handed over as pageable host arrays",
            "config": {"workload": f"{total_rays} photon segments, GJ dipole, "
                                   f"{'flat space' if params.flat else 'Schwarzschild GR'}, {args.integrator}; "
                                   "one art_propagate_host call per rank per step (H2D + kernels + D2H, SURVEY 8(d))",
                       "baseline_config": ("configs[2] (1e7 rays, sharded over the GPUs)" if args.rays == 10_000_000
                                           else ("configs[3] (1e6 GR rays, one batch)" if gr and args.rays == 1_000_000
                                                 else f"{args.rays} rays")),
                       "m_a_eV": params.mass_a, "theta_m": params.theta_m, "omega_pul": params.omega_pul,
                       "B0_G": params.B0, "rNS_km": params.rNS, "abstol": params.abstol, "reltol": params.reltol,
                       "interp_points": params.interp_points, "parallelism": f"rays sharded x{world}",
                       "host_calls_in_flight": args.inflight, "host_numa_node": numa_node,
                       "host_path": ("streamed pipeline" if streamed else
                                     "single launch" if cnt["single"] == args.steps else str(cnt)),
                       "host_path_counters": cnt, "host_path_counters_warmup": cnt_w},
            "roofline": {"bound": "fp64-valu", "achieved": fpl / (basis_ms * 1e-3) / 1e12, "peak": PEAK_FP64_TFLOPS,
                         "unit": "TFLOP/s", "frac": fpl / (basis_ms * 1e-3) / 1e12 / PEAK_FP64_TFLOPS,
                         "traffic": tr, "traffic_source": tr_src, "kernel": kname, "kernel_ms": kms,
                         "time_basis": ("the integrator launch's own duration (HIP events on its stream), mean over "
                                        "the timed passes" if args.inflight == 1 else
                                        f"wall per host call ({args.inflight} calls in flight overlap their launches)"),
                         "kernel_span_ms": float(np.mean(host_span)) if host_span else None,
                         "kernel_span_ms_each": host_span,
                         "frac_span": (fpl / (np.mean(host_span) * 1e-3) / 1e12 / PEAK_FP64_TFLOPS) if host_span else None,
                         "span_basis": "the same launches from in-kernel clock stamps (first wave start to last wave "
                                       "end, s_memrealtime at 100 MHz; art_recent_kernel_span_ms): no profiler",
                         "kernel_ms_each": host_kms,
                         "achieved_wall": fpl / (host_ms * 1e-3) / 1e12,
                         "frac_wall": fpl / (host_ms * 1e-3) / 1e12 / PEAK_FP64_TFLOPS,
                         "wall_basis": "the whole host pass (ms_per_step: H2D + kernels + D2H)",
                         "flops_per_launch": fpl, "flops_per_ray_step": fpl / host_stats["accepted"],
                         "frac_round1_flop_table": flops_per_launch(host_stats, fl_r1, args.integrator) / (kms * 1e-3)
                                                   / 1e12 / PEAK_FP64_TFLOPS,
                         "note": "FP64 VALU-bound (state in VGPRs, ~1 B of HBM per ray-step); peak = 78.6 TFLOP/s "
                                 "FP64 (vector = matrix dense peak). FLOPs from the kernel's counters x "
                                 "tools/flops.json (instrumented restatement).",
                         "hbm": {"algorithmic_bytes_per_launch": alg_bytes,
                                 "achieved_GBs": alg_bytes / (kms * 1e-3) / 1e9, "peak_GBs": PEAK_HBM_GBS,
                                 "frac": alg_bytes / (kms * 1e-3) / 1e9 / PEAK_HBM_GBS},
                         "pcie": {"h2d_bytes": in_b, "d2h_bytes": out_b,
                                  "achieved_GBs": (in_b + out_b) / (host_ms * 1e-3) / 1e9}},
            "kernel_stats": host_stats,
            "status_counts": np.bincount(host_status, minlength=5).tolist(),
            "attempts_per_ray": attempt_dist,
            "flux_hist_sum": float(flux_red["host"].sum()),
            "flux_hist": np.asarray(flux_red["host"].cpu() if hasattr(flux_red["host"], "cpu") else flux_red["host"],
                                    np.float64).reshape(-1).tolist(),
            "totals": {"rays": int(total_rays), "accepted_steps_per_pass": int(host_steps_total // args.steps)},
            "ic_sampling_s": sample_s,
        }
        if dev:
            def dev_obj(d, label):
                fpl_d = flops_per_launch(d["stats"], fl, args.integrator)
                basis = d["kernel_ms"] if d["streams"] == 1 else d["ms_per_step"]
                trd, trd_src = traffic("device")
                o = {"value": d["value"], "unit": "ray-steps/s", "ms_per_step": d["ms_per_step"],
                     "workload": label, "streams": d["streams"], "tail_donation": d["tail_donation"],
                     "roofline": {"achieved": fpl_d / (basis * 1e-3) / 1e12,
                                  "frac": fpl_d / (basis * 1e-3) / 1e12 / PEAK_FP64_TFLOPS,
                                  "kernel": "propagate_kernel<Vern6>" if args.integrator == "vern6" else
                                            "propagate_kernel<RK4>", "kernel_ms": d["kernel_ms"],
                                  "kernel_span_ms": d["kernel_span_ms"],
                                  "time_basis": ("launch duration (HIP events)" if d["streams"] == 1 else
                                                 f"wall per launch ({d['streams']} overlapping passes)"),
                                  "traffic": trd if d["streams"] == 1 else None,
                                  "traffic_source": trd_src if d["streams"] == 1 else None,
                                  "achieved_wall": fpl_d / (d["ms_per_step"] * 1e-3) / 1e12},
                     "flux_equal_host": bool(np.array_equal(d["hist"], flux_red["host"].cpu().numpy()))}
                return o
            line["device_resident"] = dev_obj(dev["one"], "inputs already in HBM, one batch per step "
                                                          "(art_propagate_device), outputs left in HBM")
            if "many" in dev:
                line["device_resident_in_flight"] = dev_obj(
                    dev["many"], f"inputs in HBM, {dev['many']['streams']} batches in flight on as many HIP streams "
                                 "(tail donation); a throughput figure, not one batch's latency")
        if world == 1 and not args.no_cpu_baseline:
            threads = int(os.environ.get("ART_CPU_THREADS", str(host_cores())))

            def sample(m):
                xs = h["x0"].reshape(3, n)[:, :m].reshape(-1).copy()
                ks = h["k0"].reshape(3, n)[:, :m].reshape(-1).copy()
                return xs, ks, h["erg"][:m].copy()
            cfg = CONFIGS[args.config] | {"integrator": 0}
            line["cpu_baseline"] = cpu_baseline(cfg, *sample(min(args.cpu_rays, n)), args.seed, threads)
            # and one core: the reference's own model is one single-threaded process per ray batch
            line["cpu_baseline"]["one_thread"] = cpu_baseline(cfg, *sample(min(args.cpu_rays_1t, n)), args.seed, 1)
            # the ForwardDiff-like restatement (the reference's per-RHS cost: three dual-number passes)
            fd = cpu_baseline(cfg, *sample(min(args.cpu_rays_oracle, n)), args.seed, threads, same_algorithm=False)
            fd["one_thread"] = cpu_baseline(cfg, *sample(min(args.cpu_rays_oracle_1t, n)), args.seed, 1,
                                            same_algorithm=False)
            line["cpu_baseline"]["forwarddiff_restatement"] = fd
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
