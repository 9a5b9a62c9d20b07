"""Dev: wall time of small art_propagate_host calls (a Julia host's per-event batches) with the
one-wave-per-ray tail mode (ART_SMALL_TAIL default) and without it (ART_SMALL_TAIL=0), flat and
GR forward roots of the configs' first rays. One JSON line per (config, n, mode)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402

for name, kw in (("flat", dict(theta_m=0.2, mass_a=1e-5, flat=True)), ("gr", dict(theta_m=0.0, mass_a=1e-6, flat=False))):
    p = A.Params(**kw)
    s = A.sample_conversion_points(p, 1024, seed=1769)
    for n in (1, 8, 64, 256, 1024):
        x, k = s["x"].reshape(3, -1)[:, :n].ravel(), s["k_init"].reshape(3, -1)[:, :n].ravel()
        args = (x, k, s["erg"][:n], -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8))
        for mode in ("tail", "lanes"):
            os.environ["ART_SMALL_TAIL"] = "1024" if mode == "tail" else "0"
            A.propagate_batch(p, *args)  # warm-up
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                r = A.propagate_batch(p, *args)
                ts.append((time.perf_counter() - t0) * 1e3)
            att = int((r["n_accept"] + r["n_reject"]).max())
            print(json.dumps({"config": name, "n": n, "mode": mode, "ms_min": min(ts), "ms_all": ts,
                              "kernel_ms": r["kernel_ms"],
                              "max_attempts": att}), flush=True)
