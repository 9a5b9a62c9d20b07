"""Dev: what predicts a ray's cost (step attempts) in the flat 1e6-ray batch? Prints the
attempt quantiles and, for a few start-point features, their rank correlation with the
attempt count and their distribution among the costliest 0.1% of rays."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
kw = json.loads(os.environ.get("COST_KW", '{"theta_m": 0.2, "mass_a": 1e-5, "flat": true}'))
p = A.Params(**kw)
eng = Engine(p)
inp = eng.forward_roots(n, seed=1769)
out = eng.propagate(inp)
att = (out["n_accept"] + out["n_reject"]).cpu().numpy().astype(np.float64)
x = inp["x0"].cpu().numpy().reshape(3, n)
k = inp["k0"].cpu().numpy().reshape(3, n)
r = np.linalg.norm(x, axis=0)
ct = x[2] / r
st = np.sqrt(np.maximum(0.0, 1.0 - ct * ct))
phi = np.arctan2(x[1], x[0])
cm, sm = np.cos(kw["theta_m"]), np.sin(kw["theta_m"])
a1 = cm * ct + sm * st * np.cos(phi)
a2 = cm * st - sm * ct * np.cos(phi)
b = 2 * a1 * ct - a2 * st
kn = k / np.linalg.norm(k, axis=0)
kr = np.sum(kn * x, axis=0) / r
# direction of B (up to B_n): 2 a1 r_hat + a2 theta_hat + a3 phi_hat -> cos(k, B)
rh = x / r
th = np.stack([ct * np.cos(phi), ct * np.sin(phi), -st])
ph = np.stack([-np.sin(phi), np.cos(phi), np.zeros(n)])
a3 = sm * np.sin(phi)
B = 2 * a1 * rh + a2 * th + a3 * ph
kB = np.abs(np.sum(kn * B, axis=0)) / np.linalg.norm(B, axis=0)
feats = {"r0": r, "|b0|": np.abs(b), "|cos theta0|": np.abs(ct), "k_r": kr, "|cos(k,B)|": kB}


def rank(v):
    o = np.argsort(v, kind="stable")
    rr = np.empty(len(v))
    rr[o] = np.arange(len(v))
    return rr


ra = rank(att)
q = np.quantile(att, [0.5, 0.9, 0.99, 0.999, 0.9999, 1.0])
top = att >= np.quantile(att, 0.999)
res = {"attempt_quantiles(50,90,99,99.9,99.99,max)": q.tolist(), "mean": float(att.mean())}
for name, v in feats.items():
    res[name] = {"spearman": float(np.corrcoef(ra, rank(v))[0, 1]),
                 "all_q10_50_90": np.quantile(v, [0.1, 0.5, 0.9]).round(4).tolist(),
                 "top0.1%_q10_50_90": np.quantile(v[top], [0.1, 0.5, 0.9]).round(4).tolist()}
# share of the total attempts held by the costliest rays
s = np.sort(att)[::-1]
res["share_top_0.1%"] = float(s[: n // 1000].sum() / s.sum())
res["share_top_1%"] = float(s[: n // 100].sum() / s.sum())
print(json.dumps(res, indent=1), flush=True)
if len(sys.argv) > 2:  # dump for offline analysis (float32 start state, attempt counts)
    np.savez_compressed(sys.argv[2], x0=x.astype(np.float32), k0=k.astype(np.float32),
                        att=att.astype(np.int32), acc=out["n_accept"].cpu().numpy().astype(np.int32))
