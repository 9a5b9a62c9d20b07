"""Development check on the GPU box: parity of libart.so against the oracle on small
seeded batches, then a first timing. Writes a JSON summary to gpurun_out/quick.json."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
import oracle as O  # noqa: E402

res = {}
for name, kw in {"flat_tm0.2": dict(theta_m=0.2, mass_a=1e-5, flat=True),
                 "gr_tm0": dict(theta_m=0.0, mass_a=1e-6, flat=False)}.items():
    p = A.Params(**kw)
    po = O.make_params(**kw)
    maxr = A.Find_Conversion_Surface(p)
    n = 256
    t = time.time()
    s = A.sample_conversion_points(p, n, seed=1769)
    ts = time.time() - t
    so = O.sample(po, maxr, 1769, 0, n)
    dx = np.abs(s["x"] - so["x"]).max()
    same_att = float(np.mean(s["attempts"] == so["attempts"]))
    # propagate the oracle's ICs on both
    r = A.propagate_batch(p, so["x"], so["k_init"], so["erg"], -np.ones(n), -30 * np.ones(n), np.ones(n, np.int8),
                          max_crossings=-1, capacity=1)
    ro = O.propagate(po, so["x"], so["k_init"], so["erg"], -1.0, -30.0, 1)
    st_agree = float(np.mean(r["status"] == ro["status"]))
    ok = r["status"] == ro["status"]
    xe, xeo = r["x_end"].reshape(3, n), ro["x_end"].reshape(3, n)
    rel = np.abs(xe - xeo).max(0) / np.linalg.norm(xeo, axis=0)
    c = ok & (ro["status"] == 1)
    pr = np.abs(r["xc_p"][c] - ro["xc_p"][c]) / np.abs(ro["xc_p"][c])
    res[name] = {"maxr": maxr, "sample_s": ts, "sample_dx_max": float(dx), "attempts_agree": same_att,
                 "status_agree": st_agree, "xend_rel_med": float(np.median(rel[ok])), "xend_rel_max": float(rel[ok].max()),
                 "P_rel_med": float(np.median(pr)) if pr.size else None, "P_rel_max": float(pr.max()) if pr.size else None,
                 "acc_gpu": float(r["n_accept"].mean()), "acc_oracle": float(ro["n_accept"].mean()),
                 "status_gpu": np.bincount(r["status"], minlength=5).tolist(),
                 "status_oracle": np.bincount(ro["status"], minlength=5).tolist(), "stats": r["stats"]}
    print(name, json.dumps(res[name]), flush=True)
    # timing on a bigger batch
    N = 1000000
    t = time.time()
    s = A.sample_conversion_points(p, N, seed=1769)
    ts = time.time() - t
    for rep in range(3):
        r = A.propagate_batch(p, s["x"], s["k_init"], s["erg"], -np.ones(N), -30 * np.ones(N), np.ones(N, np.int8))
    res[name]["timing"] = {"N": N, "sample_s": ts, "kernel_ms": r["kernel_ms"], "stats": r["stats"],
                           "ray_steps_per_s": r["stats"]["accepted"] / (r["kernel_ms"] * 1e-3)}
    print(name, "timing", json.dumps(res[name]["timing"]), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open(f"gpurun_out/quick{os.environ.get('QUICK_TAG', '')}.json", "w"), indent=1)
