"""Dev: tail donation (art_set_tail_donation) changes no result: 20k rays of several
configurations propagated with donation off and on (lanes 8, 32), every output and the
launch counters compared bit for bit. Prints one line per configuration."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

CFGS = {"flat": dict(theta_m=0.2, mass_a=1e-5, flat=True), "gr": dict(theta_m=0.0, mass_a=1e-6, flat=False),
        "scan6": dict(mass_a=1e-6, B0=2e14, omega_pul=12.566370614359172, theta_m=0.2, flat=True)}
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
bad = 0
for name, kw in CFGS.items():
    eng = Engine(A.Params(**kw))
    inp = eng.forward_roots(n, seed=1769)
    res = {}
    for lanes in (0, 8, 32):
        eng.set_tail_donation(lanes)
        out = eng.propagate(inp, max_crossings=-1)
        ms = eng.kernel_ms()
        st = A.raytracer.last_stats()
        res[lanes] = ({k: v.cpu().numpy() for k, v in out.items() if hasattr(v, "cpu")}, st, ms)
    eng.set_tail_donation(0)
    for lanes in (8, 32):
        a, b = res[0][0], res[lanes][0]
        has = a["n_cross"] > 0  # crossing slots of rays without a crossing are never written
        diff = []
        for k in a:
            x, y = a[k], b[k]
            if k.startswith("xc_"):
                x, y = x.reshape(-1, n)[:, has], y.reshape(-1, n)[:, has]
            if not np.array_equal(x, y, equal_nan=True):
                diff.append(k)
        sd = {k: (res[0][1][k], res[lanes][1][k]) for k in ("attempts", "accepted", "root_steps", "rays")
              if res[0][1][k] != res[lanes][1][k]}
        bad += bool(diff) or bool(sd)
        print(json.dumps({"config": name, "lanes": lanes, "outputs_differ": diff, "stats_differ": sd,
                          "kernel_ms_off": res[0][2], "kernel_ms_on": res[lanes][2]}), flush=True)
sys.exit(1 if bad else 0)
