"""The oracle (oracle/, test infrastructure) on single rays of a sampled batch and on 1-ulp
perturbations of their start positions: the spread of step attempts, accepted steps and end
point the reference's arithmetic itself shows for a chaotic ray, against which the GPU's
counts for the same ray are read (DESIGN.md §3, configs[3]'s longest ray 717277).
Usage: oracle_ray_sensitivity.py [ray ...]   (GR: configs[3] parameters, seed 1769)"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle as O  # noqa: E402

rays = [int(a) for a in sys.argv[1:]] or [717277]
O.build()
p = O.make_params(theta_m=0.0, mass_a=1e-6, flat=False)
mr = O.find_conversion_surface(p)
for ray in rays:
    s = O.sample(p, mr, 1769, ray, 1, nthreads=1)
    runs = []
    for k in range(7):  # unperturbed, then x, y, z one ulp up and one ulp down
        x = s["x"].copy()
        if k:
            c = (k - 1) % 3
            x[c] = np.nextafter(x[c], np.inf if k <= 3 else -np.inf)
        r = O.propagate(p, x, s["k_init"], s["erg"], -1.0, -30.0, 1, max_crossings=-1, nthreads=1)
        runs.append({"perturbed": "none" if k == 0 else f"x[{(k - 1) % 3}] {'+' if k <= 3 else '-'}1 ulp",
                     "attempts": int(r["n_accept"][0] + r["n_reject"][0]), "accepted": int(r["n_accept"][0]),
                     "status": int(r["status"][0]), "x_end": r["x_end"].tolist()})
    a = [q["attempts"] for q in runs]
    acc = [q["accepted"] for q in runs]
    print(json.dumps({"ray": ray, "config": "configs[3] GR (theta_m 0, m_a 1e-6, seed 1769)", "runs": runs,
                      "attempts_range": [min(a), max(a)], "accepted_range": [min(acc), max(acc)]}), flush=True)
