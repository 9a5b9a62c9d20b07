"""Dev: one backtrace-style propagate (flat or GR, species, n, capacity) for the library named by
ART_LIB; prints the outcome or the error. usage: exp_axn_case.py cfg species n cap"""
import json
import os
import sys
from dataclasses import replace

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes  # noqa: E402
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import _lib  # noqa: E402

if "ART_LIB" in os.environ:
    _probe = ctypes.CDLL(os.environ["ART_LIB"])
    for _name in [k for k in _lib.SIGNATURES if not hasattr(_probe, k)]:
        del _lib.SIGNATURES[_name]
cfg, species, n, cap = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
kw = dict(theta_m=0.2, mass_a=1e-5, flat=True) if cfg == "flat" else dict(theta_m=0.0, mass_a=1e-6, flat=False)
p = A.Params(**kw)
s = A.sample_conversion_points(p, n, seed=1769)
q = replace(p, B0=-p.B0) if species == 0 else p
k = -s["k_init"] if species == 0 else s["k_init"]
r = A.propagate_batch(q, s["x"], k, s["erg"], -np.ones(n), np.full(n, -30.0), np.full(n, species, np.int8),
                      max_crossings=100000 if species == 0 else -1, capacity=cap)
print(json.dumps({"lib": os.environ.get("ART_LIB", "default"), "cfg": cfg, "species": species, "n": n, "cap": cap,
                  "ok": True, "kernel_ms": r["kernel_ms"], "accepted": int(r["n_accept"].sum()),
                  "grid": r["stats"]["grid"]}), flush=True)
