"""Dev experiment: RT.propagate without callbacks (make_tree = false) on the GPU vs the
oracle in the same mode, per ray."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
import oracle as O  # noqa: E402
from adiabatic_raytracer_amd.raytracer import ART_NO_CALLBACKS  # noqa: E402

kw = dict(theta_m=0.2, mass_a=1e-5, flat=True)
po = O.make_params(**kw)
n = 128
s = O.sample(po, O.find_conversion_surface(po), 1769, 0, n)
erg = np.full(n, s["erg"][0])
p = A.Params(**kw)
for mc in (ART_NO_CALLBACKS, -1):
    g = A.propagate_batch(p, s["x"], s["k_init"], erg, -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8), max_crossings=mc)
    o = O.propagate(po, s["x"], s["k_init"], erg, -1.0, -30.0, 1, max_crossings=mc)
    xg, xo = g["x_end"].reshape(3, n), o["x_end"].reshape(3, n)
    rel = np.abs(xg - xo).max(0) / np.linalg.norm(xo, axis=0)
    print(json.dumps({"mc": mc, "pct": np.percentile(rel, [50, 90, 99]).tolist(), "status_g": np.bincount(g["status"], minlength=5).tolist(),
                      "status_o": np.bincount(o["status"], minlength=5).tolist()}))
    for i in np.argsort(-rel)[:12]:
        print(json.dumps({"ray": int(i), "rel": float(rel[i]), "st": [int(g["status"][i]), int(o["status"][i])],
                          "acc": [int(g["n_accept"][i]), int(o["n_accept"][i])], "rej": [int(g["n_reject"][i]), int(o["n_reject"][i])],
                          "r": [float(np.linalg.norm(xg[:, i])), float(np.linalg.norm(xo[:, i]))],
                          "tau": [float(g["tau_end"][i]), float(o["tau_end"][i])]}))
