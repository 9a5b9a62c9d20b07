"""Event throughput of the full pipeline, §8(f) rank 1: main_runner_tree (MainRunner.jl:354-763)
batched on the GPU against the oracle's event-by-event restatement on one host thread. The
oracle follows the reference's own model of one event at a time per process.

Each event is one sampled conversion point (find_samples_new). It then gets its backtrace
tree (axion, -B0, every crossing) and its forward photon tree. The defaults are
num_cutoff = MC_nodes = 5 and max_nodes = 50.

usage: [ART_DONATE=lanes] exp_events.py [flat|gr] [gpu event counts, comma-separated] [cpu events]
Prints one JSON line per run."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import trees  # noqa: E402

CFG = {"flat": dict(theta_m=0.2, mass_a=1e-5, flat=True), "gr": dict(theta_m=0.0, mass_a=1e-6, flat=False)}
cfg = sys.argv[1] if len(sys.argv) > 1 else "flat"
counts = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "1000,10000").split(",")]
n_cpu = int(sys.argv[3]) if len(sys.argv) > 3 else 50
p = A.Params(**CFG[cfg])
DONATE = int(os.environ.get("ART_DONATE", "-1"))  # tail donation of the forest's launches (-1: the library default)
if DONATE >= 0:
    import ctypes as C
    A._lib.load().art_set_tail_donation(C.c_int32(DONATE))

trees.main_runner_tree(p, 65)  # warm-up: library load, kernels, pools
for n in counts:
    info = {}
    t0 = time.perf_counter()
    rows = trees.main_runner_tree(p, n + 1, run_info=info)
    dt = time.perf_counter() - t0
    print(json.dumps({"config": cfg, "side": "gpu", "donate": DONATE, "events": n, "wall_s": dt, "events_per_s": n / dt,
                      "rows": int(rows.shape[0]), "f_inx": info["f_inx"]}), flush=True)

if n_cpu > 0:
    import oracle as O
    from oracle.tree import main_runner_rows
    O.build()
    po = O.make_params(**CFG[cfg])
    t0 = time.perf_counter()
    rows = main_runner_rows(po, n_cpu + 1)
    dt = time.perf_counter() - t0
    print(json.dumps({"config": cfg, "side": "cpu (oracle, 1 thread, event by event)", "events": n_cpu, "wall_s": dt,
                      "events_per_s": n_cpu / dt, "rows": int(rows.shape[0])}), flush=True)
