"""Dev: the GR workload's (configs[3]) longest rays alone. Finds the rays with the most step
attempts in the 1e6-ray GR batch, then integrates the longest one as a batch of one ray (one
lane of one wave: the latency floor of that configuration) and prints µs per attempt; with
the ART_SECTION_TIMING build (ART_LIB=...) also the lone wave's section split.
Usage: [ART_LIB=...] [TAIL_KW='{"mass_a": ...}'] exp_gr_tail.py [n] [ray]  (TAIL_KW: another
Params keyword set, e.g. a scan point)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
KW = json.loads(os.environ.get("TAIL_KW", '{"theta_m": 0.0, "mass_a": 1e-6, "flat": false}'))
eng = Engine(A.Params(**KW))
DONATE = int(os.environ.get("TAIL_DONATE", "0"))  # > 0: the ray goes to the one-wave-per-ray tail kernel
sect = any(k in os.environ.get("ART_LIB", "") for k in ("sect", "slot"))
if len(sys.argv) > 2:
    ray = int(sys.argv[2])
else:
    inp = eng.forward_roots(n, seed=1769)
    out = eng.propagate(inp)
    att = (out["n_accept"] + out["n_reject"])
    top = att.topk(8)
    print(json.dumps({"batch_kernel_ms": eng.kernel_ms(), "top_attempts": top.values.tolist(),
                      "top_rays": top.indices.tolist(), "mean_attempts": float(att.double().mean())}), flush=True)
    ray = int(top.indices[0])
inp1 = eng.forward_roots(1, seed=1769, ray_offset=ray)
eng.set_tail_donation(DONATE)
for _ in range(2):
    out1 = eng.propagate(inp1)
ms = eng.kernel_ms()
st = A.raytracer.last_stats()
a = int(out1["n_accept"][0] + out1["n_reject"][0])
line = {"ray": ray, "kernel_ms": ms, "attempts": a, "us_per_attempt": ms * 1e3 / a,
        "status": int(out1["status"][0]), "donate": DONATE, "tail": os.environ.get("ART_TAIL", "1"),
        "x_end": out1["x_end"].cpu().tolist(), "n_accept": int(out1["n_accept"][0])}
if sect:
    NAMES = ["refill etc", "stage slots", "norm/controller/cert/park", "grid pass", "fast paths", "walk", "coop pass",
             "fallback"]
    if "slot" in os.environ.get("ART_LIB", ""):
        NAMES = ["refill etc", "slot combination", "slot RHS", "slot rest", "norm/controller/cert/park", "grid pass",
                 "fast+walk+coop", "fallback"]
    v = list(st.values())[:8]
    v[6] -= 2
    tot = sum(v)
    line["sections"] = {k: round(x / tot, 4) for k, x in zip(NAMES, v)}
else:
    line["stats"] = {k: int(x) for k, x in st.items()}
print(json.dumps(line), flush=True)
