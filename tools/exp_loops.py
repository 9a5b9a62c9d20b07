import json, os, sys
sys.path.insert(0, "/root/repo")
import adiabatic_raytracer_amd as A
from adiabatic_raytracer_amd import Engine
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
for name, kw in (("flat", dict(theta_m=0.2, mass_a=1e-5, flat=True)),):
    eng = Engine(A.Params(**kw))
    inp = eng.forward_roots(n, seed=1769)
    out = eng.alloc_out(n)
    for _ in range(2):
        eng.propagate(inp, out); ms = eng.kernel_ms()
    print(json.dumps({"config": name, "kernel_ms": ms, **A.raytracer.last_stats()}), flush=True)
