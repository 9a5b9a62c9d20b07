"""Dev: where the integrator's time goes, per main-loop section, from the
ART_SECTION_TIMING build (s_memtime cycles summed over every wave's iterations; the
stats slots carry the 8 section sums). Usage: ART_LIB=.../libart_sect.so exp_sections.py [n]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

NAMES = ["refill + reload, events, finish, stores", "step size + stage slots", "error norm, controller, certificate, parking",
         "grid pass", "sign-code fast paths", "code walk", "cooperative pass", "per-lane fallback"]
if "slot" in os.environ.get("ART_LIB", ""):
    NAMES = ["refill etc", "slot combination", "slot RHS", "slot rest", "norm/controller/cert/park", "grid pass",
             "fast+walk+coop", "fallback"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
eng = Engine(A.Params(theta_m=0.2, mass_a=1e-5, flat=True))
inp = eng.forward_roots(n, seed=1769)
out = eng.alloc_out(n)
for _ in range(2):
    eng.propagate(inp, out)
ms = eng.kernel_ms()
st = list(A.raytracer.last_stats().values())[:8]
st[6] -= 2 * n  # init_kernel's RHS count shares slot 6
tot = sum(st)
print(json.dumps({"kernel_ms": ms, "sections": {k: round(v / tot, 4) for k, v in zip(NAMES, st)},
                  "cycles_total": tot}), flush=True)
