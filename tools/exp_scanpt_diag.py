"""Dev: per-ray x_end error of the GPU (ART_LIB) against the oracle at configs[4] grid point
(m_a=1e-5, B0=2e14, P=1 s), n=384, next to the oracle's own 1-ulp envelope (3 draws): the
largest errors with their rays' step and crossing counts."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import adiabatic_raytracer_amd as A  # noqa: E402
import oracle as O  # noqa: E402
from adiabatic_raytracer_amd.scan import scan_grid  # noqa: E402
from test_gpu_propagate import _rel_end, _run  # noqa: E402

O.build()
kw = [g for g in scan_grid() if g["mass_a"] == 1e-5 and g["B0"] == 2e14 and abs(g["omega_pul"] - 2 * np.pi) < 1e-12][0]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 384
g, o, o2 = _run(kw, n, oracle_lib=O)
e = _rel_end(g, o, n)
env = np.max([_rel_end(q, o, n) for q in o2], axis=0)
same = g["status"] == o["status"]
top = np.argsort(-e)[:10]
print(json.dumps({"lib": os.environ.get("ART_LIB", "default"), "p": [float(np.percentile(e, q)) for q in (50, 90, 99)],
                  "env_p": [float(np.percentile(env, q)) for q in (50, 90, 99)], "status_agree": float(same.mean()),
                  "top": [{"ray": int(i), "err": float(e[i]), "env": float(env[i]), "acc_g": int(g["n_accept"][i]),
                           "acc_o": int(o["n_accept"][i]), "st_g": int(g["status"][i]), "st_o": int(o["status"][i]),
                           "nc_g": int(g["n_cross"][i]), "nc_o": int(o["n_cross"][i])} for i in top]}), flush=True)
