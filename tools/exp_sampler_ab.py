"""Dev: samples of the library named by ART_LIB on three configurations, saved for an exact
comparison between builds. Usage: ART_LIB=... exp_sampler_ab.py OUT.npz [n]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402

n = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
cfgs = {"flat": dict(theta_m=0.2, mass_a=1e-5, flat=True), "gr": dict(theta_m=0.0, mass_a=1e-6, flat=False),
        "scan7": dict(theta_m=0.2, mass_a=1e-6, B0=2e14, omega_pul=2 * np.pi / 0.5, flat=True)}
res = {}
for name, kw in cfgs.items():
    p = A.Params(**kw)
    A.sample_conversion_points(p, 1000, seed=1769)  # warm-up
    t0 = time.perf_counter()
    s = A.sample_conversion_points(p, n, seed=1769)
    dt = time.perf_counter() - t0
    print(name, f"{dt:.3f} s", flush=True)
    for k in ("x", "k_init", "erg", "attempts"):
        res[f"{name}_{k}"] = np.asarray(s[k])
np.savez(sys.argv[1], **res)
