"""Dev: does any initial-condition feature predict a ray's step attempts (the persistent
kernel's drain tail would shrink if long rays started first)? Spearman rank correlations
on the 1e6-ray flat batch. Usage: exp_cost_predictor.py [n]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
eng = Engine(A.Params(theta_m=0.2, mass_a=1e-5, flat=True))
inp = eng.forward_roots(n, seed=1769)
out = eng.propagate(inp)
att = (out["n_accept"] + out["n_reject"]).double()
x = inp["x0"].view(3, n)
k = inp["k0"].view(3, n)
r = x.norm(dim=0)
kn = k.norm(dim=0)
feat = {"r0": r, "cos_theta": x[2] / r, "abs_cos_theta": (x[2] / r).abs(), "erg": inp["erg"], "k": kn,
        "k_radial": (x * k).sum(0) / (r * kn), "k_z": k[2] / kn, "abs_k_z": (k[2] / kn).abs(),
        "rho": x[:2].norm(dim=0), "status": out["status"].double()}


def rank(v):
    o = torch.argsort(v)
    rk = torch.empty_like(v)
    rk[o] = torch.arange(v.numel(), dtype=v.dtype, device=v.device)
    return rk


ra = rank(att)
res = {}
for name, v in feat.items():
    rv = rank(v.double())
    res[name] = float(torch.corrcoef(torch.stack([ra, rv]))[0, 1])
top = att >= torch.quantile(att[: 1 << 20], 0.99)
print(json.dumps({"spearman_vs_attempts": res, "mean_attempts": float(att.mean()),
                  "top1pct_mean_status": float(feat["status"][top].mean())}), flush=True)
