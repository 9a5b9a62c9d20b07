"""Dev: propagate outputs of the library named by ART_LIB on 20k rays of every configuration
(flat, GR, GR oblique, a scan point, the axion backtrace), saved for an exact comparison
between builds. Usage: ART_LIB=... exp_prop_ab.py OUT.npz"""
import os
import sys
from dataclasses import replace

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd.scan import scan_grid  # noqa: E402

CF = {"flat": dict(theta_m=0.2, mass_a=1e-5, flat=True), "gr": dict(theta_m=0.0, mass_a=1e-6, flat=False),
      "gr_oblique": dict(theta_m=0.2, mass_a=1e-5, flat=False), "scan7": scan_grid()[7]}
KEYS = ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept", "n_reject", "n_cross", "xc_pos", "xc_k", "xc_t",
        "xc_dw", "xc_p")
res = {}
n = 20000
for name, kw in list(CF.items()) + [("back", CF["gr"])]:
    p = A.Params(**kw)
    s = A.sample_conversion_points(p, n if name != "back" else 4000, seed=1769)
    m = s["erg"].size
    if name == "back":
        p = replace(p, B0=-p.B0)
        r = A.propagate_batch(p, s["x"], -s["k_init"], s["erg"], -np.ones(m), np.full(m, -30.0), np.zeros(m, np.int8),
                              max_crossings=100000, capacity=8)
    else:
        r = A.propagate_batch(p, s["x"], s["k_init"], s["erg"], -np.ones(m), np.full(m, -30.0), np.ones(m, np.int8))
    for k in KEYS:
        res[f"{name}_{k}"] = np.asarray(r[k])
    print(name, r["kernel_ms"], r["stats"], flush=True)
np.savez(sys.argv[1], **res)
