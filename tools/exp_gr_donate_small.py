"""Dev: GR batches between the small-batch tail mode (ART_SMALL_TAIL, 1024 rays) and the size up
to which a donation-free launch runs the 1-wave/SIMD build (ncu x 256 rays): the library default
(-1: tail donation 16 for Schwarzschild, so the 2-wave build with the continuation, the tail
kernel and graduation) against donation off (0: the 1-wave/SIMD build, no tail kernel). The
batches are forward roots of configs[3] (the first n rays of the seed-1769 batch); every
setting is timed on the same inputs, interleaved, and its outputs compared bit for bit.
One JSON line per (n, setting). ADVICE r04 (low): art_capi.cpp launch_donate."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

eng = Engine(A.Params(theta_m=0.0, mass_a=1e-6, flat=False))
sizes = [int(a) for a in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["4096", "16384", "65536"])]
reps = int(os.environ.get("REPS", "5"))
for n in sizes:
    inp = eng.forward_roots(n, seed=1769)
    outs, times = {}, {-1: [], 0: []}
    for r in range(reps + 1):
        for don in (-1, 0):
            eng.set_tail_donation(don)
            o = eng.propagate(inp)
            ms = eng.kernel_ms()
            if r > 0:
                times[don].append(ms)
            outs[don] = {k: v.cpu().numpy().copy() for k, v in o.items() if isinstance(v, torch.Tensor)}
    eng.set_tail_donation(-1)
    same = all(np.array_equal(outs[-1][k], outs[0][k], equal_nan=True) for k in outs[0])
    for don in (-1, 0):
        print(json.dumps({"n": n, "donate": don, "kernel_ms_min": min(times[don]), "kernel_ms_mean": float(np.mean(times[don])),
                          "kernel_ms_all": times[don], "bit_identical_across_settings": bool(same),
                          "max_attempts": int((outs[don]["n_accept"] + outs[don]["n_reject"]).max())}), flush=True)
