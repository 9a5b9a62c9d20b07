"""Dev (ART_TRACE build, ART_LIB=...): the per-attempt state of one ray integrated by the bulk
kernel alone (donation off) and by bulk + tail kernel (donation on); prints the first attempt
where they differ and which quantity differs first."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "gr"
ray = int(sys.argv[2]) if len(sys.argv) > 2 else 717277
KW = {"gr": dict(theta_m=0.0, mass_a=1e-6, flat=False), "flat": dict(theta_m=0.2, mass_a=1e-5, flat=True)}[cfg]
lib = A._lib.load()
lib.art_debug_trace_set.argtypes = [C.c_int]
lib.art_debug_trace_get.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int)]
eng = Engine(A.Params(**KW))
inp = eng.forward_roots(1, seed=1769, ray_offset=ray)
recs = {}
for don in (0, 16):
    eng.set_tail_donation(don)
    assert lib.art_debug_trace_set(0) == 0
    eng.propagate(inp)
    buf = np.zeros(4096 * 21)
    n = C.c_int()
    assert lib.art_debug_trace_get(buf.ctypes.data_as(C.c_void_p), 4096, C.byref(n)) == 0
    recs[don] = buf[:n.value * 21].reshape(-1, 21)
a, b = recs[0], recs[16]
names = ["kernel", "mode", "hs", "tau", "EEst2"] + [f"y{i}" for i in range(7)] + [f"kk{i}" for i in range(7)]
m = min(len(a), len(b))
first = None
for k in range(m):
    d = [names[j] for j in range(1, 21) if not (a[k, j] == b[k, j] or (np.isnan(a[k, j]) and np.isnan(b[k, j])))]
    if d:
        first = k
        print(json.dumps({"first_diff_attempt": k, "fields": d, "kernel_donated": b[k, 0],
                          "bulk": dict(zip(names, a[k].tolist())), "tail": dict(zip(names, b[k].tolist())),
                          "prev_kernel_donated": b[k - 1, 0] if k else None}), flush=True)
        break
print(json.dumps({"records": [len(a), len(b)], "first": first,
                  "kernels_donated_run": np.unique(b[:, 0]).tolist()}), flush=True)
