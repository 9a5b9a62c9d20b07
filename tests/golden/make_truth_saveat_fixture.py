"""Converged-truth saved points (TEST INFRASTRUCTURE ONLY): RT.propagate's saveat positions
(RayTracer.jl:176,383,427-444; saveNode, MainRunner.jl:17-65) for the rays of the truth fixtures
(tests/golden/make_truth_fixture.py) whose truth segment reaches ln t_end without a crossing or
the star, so that the true trajectory is the plain ODE solution from ln t0 to ln t_end.

For each such ray: scipy's DOP853 at rtol 1e-13 / atol 1e-15 on the oracle's func! restatement,
its 7th-order dense output evaluated at the interior saved times ln t0 + k (ln t_end - ln t0) /
(NTIMES - 1), k = 1 .. NTIMES - 2, and the positions back-transformed to Cartesian km
(RayTracer.jl:427-444). Writes tests/golden/truth_saveat_{case}.npz (ray indices into the truth
fixture, the times and the positions).

Regenerate (8 processes, about a minute):  python tests/golden/make_truth_saveat_fixture.py
"""
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_truth_fixture as MT  # noqa: E402

O = MT.O
NTIMES = 5
CASES = ("flat", "gr")


def saved_points(args):
    from scipy.integrate import DOP853
    kw, x0, k0, erg, times = args
    p = O.make_params(**kw)
    u0 = O.initial_state(p, x0, k0, erg, -1.0)
    sol = DOP853(lambda t, y: O.rhs(p, 1, y.copy(), t, erg), -30.0, u0, p.ln_t_end, rtol=MT.RTOL, atol=MT.ATOL)
    pts = np.full((3, len(times)), np.nan)
    j = 0
    while sol.status == "running" and j < len(times):
        sol.step()
        if sol.status == "failed":
            break
        dense = sol.dense_output()
        while j < len(times) and times[j] <= sol.t:
            pts[:, j] = MT._back_transform(p, dense(times[j]), erg)[0]
            j += 1
    return pts


def make(case, procs=8):
    z = np.load(os.path.join(HERE, f"truth_{case}.npz"))
    kw = {k[len("params_"):]: (z[k].item() if z[k].ndim == 0 else z[k]) for k in z.files if k.startswith("params_")}
    kw = {k: (bool(v) if k == "flat" else float(v)) for k, v in kw.items()}
    p = O.make_params(**kw)
    n = z["erg"].size
    rays = np.flatnonzero(z["status"] == MT.ST_SUCCESS)
    times = -30.0 + (p.ln_t_end + 30.0) * np.arange(1, NTIMES - 1) / (NTIMES - 1)
    x0, k0 = z["x0"].reshape(3, n), z["k0"].reshape(3, n)
    with Pool(procs) as pool:
        pts = pool.map(saved_points, [(kw, x0[:, i].copy(), k0[:, i].copy(), float(z["erg"][i]), times) for i in rays],
                       chunksize=1)
    pts = np.stack(pts, axis=-1)  # (3, NTIMES - 2, rays)
    np.savez_compressed(os.path.join(HERE, f"truth_saveat_{case}.npz"), rays=rays, times=times, ntimes=NTIMES, pos=pts)
    print(f"{case}: {rays.size} rays, {np.isnan(pts).any(axis=(0, 1)).sum()} without every point", flush=True)


if __name__ == "__main__":
    O.build()
    for c in sys.argv[1:] or CASES:
        make(c)
