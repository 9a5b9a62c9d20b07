"""Dev: the ART_COUNT_SUB build's counters on the flat and GR 1e6 batches: what the steps the
scan certificate leaves uncertified are. Usage: ART_LIB=.../libart_sub.so"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
NAMES = ["uncertified", "all_pos", "all_neg_e2_fail", "all_pos_near_miss", "all_neg", "sign_change", "all_neg_near_miss"]
for name, kw in (("flat", dict(theta_m=0.2, mass_a=1e-5, flat=True)), ("gr", dict(theta_m=0.0, mass_a=1e-6, flat=False))):
    eng = Engine(A.Params(**kw))
    inp = eng.forward_roots(n, seed=1769)
    out = eng.propagate(inp)
    eng.kernel_ms()
    v = list(A.raytracer.last_stats().values())
    st = v[:6] + [v[7]]  # (slot 6 holds init_kernel's RHS count)
    acc = int(out["n_accept"].sum().item())
    print(json.dumps({"config": name, "accepted": acc, **dict(zip(NAMES, st))}), flush=True)
