"""Dev: the ART_COUNT_PASSES build's wave-level counters (main iterations, grid passes,
iterations with a grid pass, cooperative passes, refilling iterations, iterations with a code
walk, fallback-loop iterations) on the flat 1e7 batch and the GR 1e6 batch.
Usage: ART_LIB=.../libart_passes.so exp_passes.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

NAMES = ["main_it", "grid_passes", "grid_iters", "coop_passes", "refill_iters", "walk_iters", "fallback_it"]
for name, n, kw in (("flat", 10_000_000, dict(theta_m=0.2, mass_a=1e-5, flat=True)),
                    ("gr", 1_000_000, dict(theta_m=0.0, mass_a=1e-6, flat=False))):
    eng = Engine(A.Params(**kw))
    inp = eng.forward_roots(n, seed=1769)
    out = eng.propagate(inp)
    eng.kernel_ms()
    v = list(A.raytracer.last_stats().values())
    st = v[:6] + [v[7]]  # (slot 6 holds init_kernel's RHS count)
    d = dict(zip(NAMES, st))
    d = {k: v / d["main_it"] if k != "main_it" else v for k, v in d.items()}
    print(json.dumps({"config": name, **d}), flush=True)
