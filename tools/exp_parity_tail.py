"""Dev experiment: the rays behind a parity test's tail (GPU vs oracle x_end error above
1e-4), next to the oracle's own sensitivity to 1-ulp perturbations of the start (3 runs)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
import oracle as O  # noqa: E402
from adiabatic_raytracer_amd.scan import scan_grid  # noqa: E402

pt = int(sys.argv[1]) if len(sys.argv) > 1 else 31
n = int(sys.argv[2]) if len(sys.argv) > 2 else 384
kw = scan_grid()[pt]
po = O.make_params(**kw)
s = O.sample(po, O.find_conversion_surface(po), 1769, 0, n)
p = A.Params(**kw)
g = A.propagate_batch(p, s["x"], s["k_init"], s["erg"], -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8))
o = O.propagate(po, s["x"], s["k_init"], s["erg"], -1.0, -30.0, 1)
rel = lambda a, b: np.abs(a["x_end"].reshape(3, n) - b["x_end"].reshape(3, n)).max(0) / np.linalg.norm(  # noqa: E731
    b["x_end"].reshape(3, n), axis=0)
eg = rel(g, o)
eo = []
for sd in (1769, 1, 2):
    ulp = np.random.default_rng(sd).choice([-1.0, 1.0], s["x"].shape) * 2.2e-16
    o2 = O.propagate(po, s["x"] * (1.0 + ulp), s["k_init"], s["erg"], -1.0, -30.0, 1)
    eo.append(rel(o2, o))
eo = np.array(eo)
print(json.dumps({"point": pt, "kw": kw, "gpu_pct": np.percentile(eg, [50, 90, 99]).tolist(),
                  "oracle_pct": [np.percentile(e, [50, 90, 99]).tolist() for e in eo]}))
for i in np.flatnonzero(eg > 1e-4):
    print(json.dumps({"ray": int(i), "err": float(eg[i]), "oracle_errs": eo[:, i].tolist(), "status": [int(g["status"][i]), int(o["status"][i])],
                      "n_acc": [int(g["n_accept"][i]), int(o["n_accept"][i])], "n_rej": [int(g["n_reject"][i]), int(o["n_reject"][i])],
                      "r_end": float(np.linalg.norm(o["x_end"].reshape(3, n)[:, i]))}))
