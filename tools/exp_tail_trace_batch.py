"""Dev (ART_TRACE build): find the rays of a batch whose result differs between the undonated
run and the donated run (bulk + packed continuation + tail kernel), then trace the first such
ray in both runs and print the first attempt that differs."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "flat"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8000
KW = {"gr": dict(theta_m=0.0, mass_a=1e-6, flat=False), "flat": dict(theta_m=0.2, mass_a=1e-5, flat=True)}[cfg]
lib = A._lib.load()
lib.art_debug_trace_set.argtypes = [C.c_int]
lib.art_debug_trace_get.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int)]
eng = Engine(A.Params(**KW))
inp = eng.forward_roots(n, seed=1769)


def run(don, trace=-1):
    eng.set_tail_donation(don)
    assert lib.art_debug_trace_set(trace) == 0
    out = eng.propagate(inp)
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 21)
    m = C.c_int()
    assert lib.art_debug_trace_get(buf.ctypes.data_as(C.c_void_p), 4096, C.byref(m)) == 0
    return {k: v.cpu().numpy() for k, v in out.items() if hasattr(v, "cpu")}, buf[:m.value * 21].reshape(-1, 21)


a, _ = run(0)
b, _ = run(16)
bad = np.nonzero((a["x_end"].reshape(3, n) != b["x_end"].reshape(3, n)).any(0) | (a["n_accept"] != b["n_accept"]))[0]
print(json.dumps({"rays_differing": int(bad.size), "first": bad[:10].tolist()}), flush=True)
names = ["kernel", "mode", "hs", "tau", "EEst2"] + [f"y{i}" for i in range(7)] + [f"kk{i}" for i in range(7)]
for r in bad[:3]:
    _, ta = run(0, int(r))
    _, tb = run(16, int(r))
    m = min(len(ta), len(tb))
    # bracket records (kernel 10 / 11: [ip, last_j, last_c, i_cg, t_int, lc_ok, th_ip] in y) side by side
    ra, rb = ta[ta[:, 0] >= 10], tb[tb[:, 0] >= 10]
    for k in range(min(len(ra), len(rb))):
        if not np.array_equal(ra[k, 5:12], rb[k, 5:12]):
            print(json.dumps({"ray": int(r), "bracket_diff": k, "bulk": ra[k, :12].tolist(), "tail": rb[k, :12].tolist()}),
                  flush=True)
            break
    ta, tb = ta[ta[:, 0] < 10], tb[tb[:, 0] < 10]
    m = min(len(ta), len(tb))
    first = None
    for k in range(m):
        d = [names[j] for j in range(1, 21) if not (ta[k, j] == tb[k, j] or (np.isnan(ta[k, j]) and np.isnan(tb[k, j])))]
        if d:
            first = k
            print(json.dumps({"ray": int(r), "first_diff_attempt": k, "fields": d, "records": [len(ta), len(tb)],
                              "kernels_b_until_k": tb[:k + 1, 0].tolist(), "modes_b": tb[max(0, k - 3):k + 1, 1].tolist(),
                              "bulk": dict(zip(names, ta[k].tolist())), "tail": dict(zip(names, tb[k].tolist()))}), flush=True)
            break
    if first is None:
        print(json.dumps({"ray": int(r), "records": [len(ta), len(tb)], "note": "traces equal",
                          "end_a": a["x_end"].reshape(3, n)[:, r].tolist(), "end_b": b["x_end"].reshape(3, n)[:, r].tolist(),
                          "status": [int(a["status"][r]), int(b["status"][r])], "acc": [int(a["n_accept"][r]), int(b["n_accept"][r])],
                          "kernels_b": np.unique(tb[:, 0]).tolist(), "last_b": tb[-1].tolist(), "last_a": ta[-1].tolist()}),
              flush=True)
