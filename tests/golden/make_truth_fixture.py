"""Converged-truth fixtures for the forward segment (TEST INFRASTRUCTURE ONLY).

The reference (Julia, OrdinaryDiffEq, ForwardDiff) cannot run here and ships no fixtures,
so the HIP engine's physics outputs are pinned to a converged solution of the reference's
equations instead of to the reference's own numbers:

* the ODE is `func!` (RayTracer.jl:71-91) as restated by the oracle (oracle_rhs, whose
  gradients are checked against finite differences in tests/test_oracle.py);
* the integrator is scipy's DOP853 (an implementation independent of this build's Vern6)
  at rtol 1e-13 / atol 1e-15 with its 7th-order dense output;
* the resonance scan follows ContinuousCallback(rootfind=true, interp_points=50)
  (RayTracer.jl:357-358): the condition (`condition`, :254-298) at 50 points of every TRUTH
  step's dense output, the first sign change bracketed and solved by brentq on the dense
  output, and `affect!` (:301-350) applied as the reference does (skip the start point on
  the first call, skip r < 1.01 rNS, terminate at the first recorded crossing for a forward
  segment, max_crossings = -1, MainRunner.jl:128,182);
* `cb_r` (:352-368) becomes its continuous limit: the ray ends when r reaches 1.01 rNS
  (below it the RHS is zero, :86, so the true trajectory is frozen there);
* P_nonAD at the crossing is `get_Prob_nonAD` (MainRunner.jl:67-124) on the truth crossing.

Rays: the forward-tree roots of the restated find_samples_new (seed 1769) for the flat,
GR, oblique-GR configurations and one configs[4] scan point; 1024 per configuration.
The fixtures hold the inputs (x0, k0, erg) and, per ray, the truth status, crossing
(x, k, t, Δω, P) or end state (x, k, u7), and the 50-bin radiated flux (plot/flux.py:38-48
over [-π, π), unit weights, non-crossing rays ending outside 1.1 rNS, MainRunner.jl:200-207).

Regenerate (8 processes, a few minutes):  python tests/golden/make_truth_fixture.py
"""
import ctypes as C
import math
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle as O  # noqa: E402

RTOL, ATOL = 1e-13, 1e-15
INTERP_POINTS = 50
MAX_TRUTH_STEPS = 400_000
N_RAYS = 1024
NBINS = 50

# configs: flat and GR are BASELINE configs[0..2] and [3] (tests/conftest.py CONFIGS); the scan
# point is configs[4]'s (m_a, B0, P) = (5e-6 eV, 5e13 G, 0.5 s), θm = 0.2, flat (scan.scan_grid)
CASES = {
    "flat": dict(theta_m=0.2, mass_a=1e-5, flat=True),
    "gr": dict(theta_m=0.0, mass_a=1e-6, flat=False),
    "gr_oblique": dict(theta_m=0.2, mass_a=1e-5, flat=False),
    "scan": dict(theta_m=0.2, mass_a=5e-6, B0=5e13, omega_pul=2.0 * math.pi / 0.5, flat=True),
}

ST_SUCCESS, ST_CROSSING, ST_HIT_NS, ST_TRUTH_FAILED = 0, 1, 2, -1


def _back_transform(p, u, erg):
    x, k = np.zeros(3), np.zeros(3)
    pd = C.POINTER(C.c_double)
    O.lib().oracle_back_transform(C.byref(p), np.ascontiguousarray(u).ctypes.data_as(pd), erg,
                                  x.ctypes.data_as(pd), k.ctypes.data_as(pd))
    return x, k


def truth_ray(args):
    """One forward segment to convergence. Returns a dict of the ray's truth outputs."""
    from scipy.integrate import DOP853
    from scipy.optimize import brentq
    kw, x0, k0, erg = args
    p = O.make_params(**kw)
    u0 = O.initial_state(p, x0, k0, erg, -1.0)
    tau0, tend = -30.0, p.ln_t_end
    rcut = 1.01 * p.rNS

    def fun(t, y):
        return O.rhs(p, 1, y.copy(), t, erg)  # a copy: the in-place clamp (:531) stays local

    def cond(t, y):
        return O.condition(p, y, t)

    sol = DOP853(fun, tau0, u0, tend, rtol=RTOL, atol=ATOL)
    out = dict(status=ST_TRUTH_FAILED, steps=0, xc=np.full(3, np.nan), kc=np.full(3, np.nan), tc=np.nan,
               dwc=np.nan, pc=np.nan, x_end=np.full(3, np.nan), k_end=np.full(3, np.nan), u7_end=np.nan,
               tau_end=np.nan)
    if u0[0] < rcut:  # starts inside 1.01 rNS: the RHS is zero there (:86), cb_r ends it
        out.update(status=ST_HIT_NS, tau_end=tau0, u7_end=u0[6])
        out["x_end"], out["k_end"] = _back_transform(p, u0, erg)
        return out
    c_prev = cond(tau0, u0)
    s_prev = 0 if math.isnan(c_prev) else int(np.sign(c_prev))
    t_prev = tau0
    count = 0  # affect!'s callback_count (records only)
    while sol.status == "running" and out["steps"] < MAX_TRUTH_STEPS:
        sol.step()
        out["steps"] += 1
        if sol.status == "failed":
            if sol.y[0] <= rcut + 1e-8:
                # the step size collapsed on the RHS's cut at r = 1.01 rNS (:86), where the true
                # ray freezes: it reached the star
                out.update(status=ST_HIT_NS, tau_end=sol.t, u7_end=sol.y[6])
                out["x_end"], out["k_end"] = _back_transform(p, sol.y, erg)
            return out
        dense = sol.dense_output()
        ts = np.linspace(sol.t_old, sol.t, INTERP_POINTS)[1:]
        ys = dense(ts)
        for j, t in enumerate(ts):
            y = ys[:, j]
            if y[0] <= rcut:  # cb_r's continuous limit: the true ray stops at 1.01 rNS
                tr = brentq(lambda tt: dense(tt)[0] - rcut, t_prev, t, xtol=1e-15, rtol=1e-15)
                ur = dense(tr)
                out.update(status=ST_HIT_NS, tau_end=tr, u7_end=ur[6])
                out["x_end"], out["k_end"] = _back_transform(p, ur, erg)
                return out
            c = cond(t, y)
            if math.isnan(c):
                s_prev = 0
                t_prev = t
                continue
            s = int(np.sign(c))
            if s_prev != 0 and s != 0 and s != s_prev:
                tr = brentq(lambda tt: cond(tt, dense(tt)), t_prev, t, xtol=1e-15, rtol=1e-15)
                ur = dense(tr)
                xc, kc = _back_transform(p, ur, erg)
                skip = False
                if count == 0:  # affect!: a crossing at the start point (:303-314)
                    skip = bool(np.all(np.abs(xc) < np.abs(x0) * 1.0001) and np.all(np.abs(xc) > np.abs(x0) / 1.0001))
                if not skip and np.linalg.norm(xc) < rcut:  # :322-324
                    skip = True
                if not skip:
                    dwc = ur[6] / erg
                    pc = O.get_prob_nonad(p, xc, kc, np.array([erg * abs(dwc)]))[0]
                    out.update(status=ST_CROSSING, xc=xc, kc=kc, tc=math.exp(tr), dwc=dwc, pc=pc, tau_end=tr)
                    return out
            if s != 0:
                s_prev = s
            t_prev = t
    if sol.status == "finished":
        u = sol.y
        out.update(status=ST_SUCCESS, tau_end=sol.t, u7_end=u[6])
        out["x_end"], out["k_end"] = _back_transform(p, u, erg)
    return out


def flux(status, x_end, k_end, rNS, nbins=NBINS):
    """plot/flux.py:38-48 over [-π, π): unit weights, is_final rays (MainRunner.jl:200-207)."""
    sel = (status != ST_CROSSING) & (status != ST_TRUTH_FAILED) & (np.linalg.norm(x_end, axis=0) > 1.1 * rNS)
    phi = np.arctan2(k_end[1, sel], k_end[0, sel])
    return np.histogram(phi, nbins, range=(-np.pi, np.pi))[0].astype(np.float64)


def make(name, kw, n=N_RAYS, procs=8):
    p = O.make_params(**kw)
    maxr = O.find_conversion_surface(p)
    s = O.sample(p, maxr, 1769, 0, n, nthreads=procs)
    x0, k0 = s["x"].reshape(3, n), s["k_init"].reshape(3, n)
    t = time.time()
    with Pool(procs) as pool:
        res = pool.map(truth_ray, [(kw, x0[:, i].copy(), k0[:, i].copy(), float(s["erg"][i])) for i in range(n)],
                       chunksize=1)
    st = np.array([r["status"] for r in res], np.int32)
    arr = {k: np.stack([r[k] for r in res], axis=-1) for k in ("xc", "kc", "x_end", "k_end")}
    sc = {k: np.array([r[k] for r in res]) for k in ("tc", "dwc", "pc", "u7_end", "tau_end", "steps")}
    hist = flux(st, arr["x_end"], arr["k_end"], p.rNS)
    np.savez_compressed(
        os.path.join(HERE, "truth_" + name + ".npz"), x0=s["x"], k0=s["k_init"], erg=s["erg"], max_r=maxr,
        status=st, xc_pos=arr["xc"].reshape(-1), xc_k=arr["kc"].reshape(-1), xc_t=sc["tc"], xc_dw=sc["dwc"],
        xc_p=sc["pc"], x_end=arr["x_end"].reshape(-1), k_end=arr["k_end"].reshape(-1), u7_end=sc["u7_end"],
        tau_end=sc["tau_end"], truth_steps=sc["steps"], flux=hist, rtol=RTOL, atol=ATOL,
        interp_points=INTERP_POINTS, **{"params_" + k: v for k, v in kw.items()})
    print(f"{name}: {n} rays in {time.time() - t:.0f} s; status counts {np.bincount(st + 1, minlength=4)} "
          f"(failed, success, crossing, hit NS); truth steps median {np.median(sc['steps']):.0f} "
          f"max {sc['steps'].max()}", flush=True)


if __name__ == "__main__":
    O.build()
    names = sys.argv[1:] or list(CASES)
    for nm in names:
        make(nm, CASES[nm])
