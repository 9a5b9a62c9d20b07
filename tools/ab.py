"""Dev A/B timing of the propagate kernel for the library named by ART_LIB: 1e6-ray (argv[1])
batches of the flat (configs[1]) and GR (configs[3]) workloads (argv[2]: only one of them).
One JSON line per config; kernel_ms is the best of the timed launches after the first."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes  # noqa: E402
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine, _lib  # noqa: E402

# older builds under comparison may predate entry points this tree binds: drop those from the
# signature table here (dev tool only; the product loader stays strict)
if "ART_LIB" in os.environ:
    _probe = ctypes.CDLL(os.environ["ART_LIB"])
    for _name in [k for k in _lib.SIGNATURES if not hasattr(_probe, k)]:
        del _lib.SIGNATURES[_name]

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
only = sys.argv[2] if len(sys.argv) > 2 else None  # "flat" or "gr"
for name, kw in (("flat", dict(theta_m=0.2, mass_a=1e-5, flat=True)), ("gr", dict(theta_m=0.0, mass_a=1e-6, flat=False))):
    if only and name != only:
        continue
    eng = Engine(A.Params(**kw))
    if "ART_AB_DONATE" in os.environ:  # tail donation lanes (default: the library's, by geometry)
        eng.set_tail_donation(int(os.environ["ART_AB_DONATE"]))
    inp = eng.forward_roots(n, seed=1769)
    out = eng.alloc_out(n)
    ms = []
    for _ in range(3 if name == "flat" else 2):
        eng.propagate(inp, out)
        ms.append(eng.kernel_ms())
    ms[-1] = min(ms[1:])
    st = A.raytracer.last_stats()
    att = (out["n_accept"] + out["n_reject"]).max().item()
    print(json.dumps({"lib": os.environ.get("ART_LIB", "default"), "config": name, "n": n, "kernel_ms": ms[-1],
                      "donate": os.environ.get("ART_AB_DONATE", "default"),
                      "accepted": st["accepted"], "scan_evals": st["scan_evals"], "interp_evals": st["interp_evals"],
                      "max_attempts": att, "ray_steps_per_s": st["accepted"] / ms[-1] * 1e3}), flush=True)
