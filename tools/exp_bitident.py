"""Dev: the outputs of one library build on fixed workloads (flat and GR forward segments on the
device path, the streamed host path, sampled forward roots), saved to an npz, so two builds
(ART_LIB) can be compared bit for bit:  exp_bitident.py OUT.npz  /  exp_bitident.py --cmp A.npz B.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if sys.argv[1] == "--cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
    print({"keys": len(a.files), "differ": bad})
    sys.exit(1 if bad else 0)

import torch  # noqa: E402

import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

res = {}
for name, kw, n in (("flat", dict(theta_m=0.2, mass_a=1e-5, flat=True), 200_000),
                    ("gr", dict(theta_m=0.0, mass_a=1e-6, flat=False), 50_000),
                    ("gro", dict(theta_m=0.2, mass_a=1e-5, flat=False), 50_000)):
    eng = Engine(A.Params(**kw))
    inp = eng.forward_roots(n, seed=1769)
    out = eng.propagate(inp, max_crossings=-1)
    torch.cuda.synchronize()
    for k in ("x0", "k0", "erg"):
        res[f"{name}_in_{k}"] = inp[k].cpu().numpy()
    for k in ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept", "n_reject", "xc_p", "xc_pos"):
        res[f"{name}_dev_{k}"] = out[k].cpu().numpy()
    if os.environ.get("BITIDENT_DEVICE_ONLY"):
        continue
    h = A.propagate_batch(A.Params(**kw), res[f"{name}_in_x0"], res[f"{name}_in_k0"], res[f"{name}_in_erg"],
                          -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8), flux_nbins=50)
    for k in ("x_end", "k_end", "u7_end", "status", "n_accept", "xc_p", "flux"):
        res[f"{name}_host_{k}"] = h[k]
np.savez(sys.argv[1], **res)
print("wrote", sys.argv[1], len(res))
