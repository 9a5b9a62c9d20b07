"""Dev: where one main_runner_tree run's wall goes (sampling, event weight, backtrace forest,
forward forest), GR configs[3] physics by default. usage: exp_event_split.py [events] [flat|gr]"""
import json
import os
import sys
import time
from dataclasses import replace

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd.raytracer import event_weight  # noqa: E402
from adiabatic_raytracer_amd.trees import grow_trees  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
cfg = sys.argv[2] if len(sys.argv) > 2 else "gr"
kw = dict(theta_m=0.2, mass_a=1e-5, flat=True) if cfg == "flat" else dict(theta_m=0.0, mass_a=1e-6, flat=False)
p = A.Params(**kw)
for rep in range(2):
    t = [time.perf_counter()]
    s = A.sample_conversion_points(p, n, seed=1769)
    t.append(time.perf_counter())
    w = event_weight(p, s["x"], s["k_init"], s["vifty"])
    t.append(time.perf_counter())
    x, k = s["x"].reshape(3, n).T, s["k_init"].reshape(3, n).T
    b = grow_trees(replace(p, B0=-p.B0), x, -k, s["erg"], 0, num_cutoff=0, splittings_cutoff=100000, crossing_cap=256)
    t.append(time.perf_counter())
    f = grow_trees(p, x, k, s["erg"], 1)
    t.append(time.perf_counter())
    d = np.diff(t)
    print(json.dumps({"config": cfg, "events": n, "sample_s": d[0], "weight_s": d[1], "backtrace_s": d[2],
                      "forward_s": d[3], "forward_nodes": int(len(f[0])), "max_count": int(f[1].max())}), flush=True)
