"""Dev: bit-level fingerprint of one library's flat 1e6/1e7 run (ART_LIB): checksums of the
sampled inputs and of every propagate output, per launch (A/B builds meant to be identical)."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes  # noqa: E402
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine, _lib  # noqa: E402

if "ART_LIB" in os.environ:
    _probe = ctypes.CDLL(os.environ["ART_LIB"])
    for _name in [k for k in _lib.SIGNATURES if not hasattr(_probe, k)]:
        del _lib.SIGNATURES[_name]


def h(t):
    return hashlib.sha256(t.contiguous().cpu().numpy().tobytes()).hexdigest()[:12]


n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
cfg = sys.argv[2] if len(sys.argv) > 2 else "flat"
kw = dict(theta_m=0.2, mass_a=1e-5, flat=True) if cfg == "flat" else dict(theta_m=0.0, mass_a=1e-6, flat=False)
eng = Engine(A.Params(**kw))
inp = eng.forward_roots(n, seed=1769)
res = {"lib": os.environ.get("ART_LIB", "default"), "n": n, "cfg": cfg, "in": h(inp["x0"]) + h(inp["k0"])}
for rep in range(2):
    out = eng.alloc_out(n)
    eng.propagate(inp, out)
    res[f"out{rep}"] = "".join(h(out[k])[:6] for k in ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept"))
    res[f"acc{rep}"] = int(out["n_accept"].sum())
print(json.dumps(res), flush=True)
