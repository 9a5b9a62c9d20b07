"""Dev: the ART_COUNT_SUB build's counters on the flat 1e6 batch (uncertified steps, uniform
7-point sub-intervals among them, uniform whole steps). Usage: ART_LIB=.../libart_sub.so"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
for name, kw in (("flat", dict(theta_m=0.2, mass_a=1e-5, flat=True)), ("gr", dict(theta_m=0.0, mass_a=1e-6, flat=False))):
    eng = Engine(A.Params(**kw))
    inp = eng.forward_roots(n, seed=1769)
    out = eng.propagate(inp)
    eng.kernel_ms()
    st = A.raytracer.last_stats()
    print(json.dumps({"config": name, "accepted": st["accepted"], "cert_steps": st["cert_steps"],
                      "uncertified": st["root_steps"], "uniform_subintervals": st["scan_evals"],
                      "uniform_pos_steps": st["interp_evals"], "uniform_neg_steps": st["rays"]}), flush=True)
