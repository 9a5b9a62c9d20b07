"""The product's physics header (art_core.h, hand-derived analytic gradients) compiled for
the host, checked against the oracle's dual-number restatement on random states for every
configuration: func!/func_axion! (RayTracer.jl:71-123), hamiltonian (:530-556), the
resonance condition (:254-298), initial/back transforms (:179-216, :393-416), the
conversion probability (MainRunner.jl:67-124) and the sampler condition (:1547-1583).
Tolerances: 1e-11 relative to each component's scale (FP64 rounding of different but
equivalent formulas); the compact sincos within 1 ulp of glibc."""
import os
import sys

import numpy as np
import pytest

from conftest import CONFIGS, random_states

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import corecheck as cc  # noqa: E402

ERG = 1.0000002692622573e-05


def test_sincos_within_one_ulp():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-200, 200, 200000), rng.uniform(-1, 1, 200000), np.linspace(-7, 7, 10001)])
    s, c = cc.sincos(x)
    rs, rc = np.sin(x), np.cos(x)
    us = np.spacing(np.abs(rs))
    uc = np.spacing(np.abs(rc))
    assert np.max(np.abs(s - rs) / us) <= 1.0
    assert np.max(np.abs(c - rc) / uc) <= 1.0


def test_exp_fma_within_one_ulp():
    """exp_fma (the device's e^x for ln t and the controller) against libm."""
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(-700, 700, 200000), rng.uniform(-30, 5, 200000),
                        rng.uniform(-1e-3, 1e-3, 20000), np.linspace(-2, 2, 10001), [0.0, -0.0]])
    y, ref = cc.exp_fma(x), np.exp(x)
    assert np.max(np.abs(y - ref) / np.spacing(ref)) <= 1.0


def test_log_fma_within_two_ulp():
    """log_fma (the controller's ln EEst²) against libm, normals and subnormals."""
    rng = np.random.default_rng(2)
    x = np.concatenate([10.0 ** rng.uniform(-300, 300, 200000), rng.uniform(0.5, 2.0, 200000),
                        1.0 + rng.uniform(-1e-6, 1e-6, 20000), [1.0, 2.0, 0.5, 5e-324, 1e-310]])
    y, ref = cc.log_fma(x), np.log(x)
    err = np.abs(y - ref) / np.spacing(np.maximum(np.abs(ref), 1e-300))
    assert np.max(err[ref != 0]) <= 2.0
    assert cc.log_fma(np.array([1.0]))[0] == 0.0


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
@pytest.mark.parametrize("species", [1, 0])
@pytest.mark.parametrize("b0sign", [1.0, -1.0])  # main_runner_tree backtraces with -B0 (:585)
def test_rhs(cfg, species, b0sign, oracle_lib):
    p = oracle_lib.make_params(B0=1e14 * b0sign, **CONFIGS[cfg])
    U, tau = random_states(400, seed=3 + species, rmin=9.5)
    for i in range(U.shape[1]):
        a = cc.rhs(p, species, U[:, i], tau[i], ERG)
        b = oracle_lib.rhs(p, species, U[:, i], tau[i], ERG)
        scale = np.maximum(np.abs(b), np.abs(b).max() * 1e-6) + 1e-300
        assert np.all(np.abs(a - b) <= 1e-11 * scale), (cfg, i, a, b)


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_boundary_layer_rhs(cfg, oracle_lib):
    kw = dict(CONFIGS[cfg], bndry_lyr=3.0)
    p = oracle_lib.make_params(**kw)
    U, tau = random_states(200, seed=9)
    for i in range(U.shape[1]):
        a = cc.rhs(p, 1, U[:, i], tau[i], ERG)
        b = oracle_lib.rhs(p, 1, U[:, i], tau[i], ERG)
        scale = np.maximum(np.abs(b), np.abs(b).max() * 1e-6) + 1e-300
        assert np.all(np.abs(a - b) <= 1e-10 * scale), (cfg, i, a, b)


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
@pytest.mark.parametrize("iso", [False, True])
@pytest.mark.parametrize("b0sign", [1.0, -1.0])  # main_runner_tree backtraces with -B0 (:585)
def test_condition(cfg, iso, b0sign, oracle_lib):
    p = oracle_lib.make_params(isotropic=iso, B0=1e14 * b0sign, **CONFIGS[cfg])
    U, tau = random_states(400, seed=5, rmin=9.5)
    for i in range(U.shape[1]):
        a, b = cc.condition(p, U[:, i], tau[i]), oracle_lib.condition(p, U[:, i], tau[i])
        assert np.isnan(a) == np.isnan(b)
        if not np.isnan(b):
            assert abs(a - b) <= 1e-10 * (abs(b) + 1e-3), (i, a, b)


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
@pytest.mark.parametrize("b0sign", [1.0, -1.0])  # main_runner_tree backtraces with -B0 (:585)
def test_hamiltonian(cfg, b0sign, oracle_lib):
    p = oracle_lib.make_params(B0=1e14 * b0sign, **CONFIGS[cfg])
    U, tau = random_states(300, seed=13, rmin=9.0)  # r < rNS exercises the clamp (RayTracer.jl:531)
    for i in range(U.shape[1]):
        x, k, T, E = U[0:3, i], U[3:6, i] * ERG, np.exp(tau[i]), -U[6, i]
        h1, gx1, gk1, gT1 = cc.hamiltonian(p, x, k, T, E)
        h2, gx2, gk2, gT2 = oracle_lib.hamiltonian(p, x, k, T, E)
        assert abs(h1 - h2) <= 1e-11 * E * E
        for a, b in ((gx1, gx2), (gk1, gk2)):
            assert np.all(np.abs(a - b) <= 1e-10 * (np.abs(b).max() + 1e-300))
        assert abs(gT1 - gT2) <= 1e-10 * (abs(gT2) + 1e-3 * np.abs(gx2).max() + 1e-300)


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
@pytest.mark.parametrize("b0sign", [1.0, -1.0])  # main_runner_tree backtraces with -B0 (:585)
def test_transforms_and_probability(cfg, b0sign, oracle_lib):
    p = oracle_lib.make_params(**CONFIGS[cfg])
    s = oracle_lib.sample(p, oracle_lib.find_conversion_surface(p), 1769, 0, 64, nthreads=1)
    n = 64
    for i in range(n):
        x, k, e = s["x"].reshape(3, n)[:, i], s["k_init"].reshape(3, n)[:, i], s["erg"][i]
        u1, u2 = cc.initial_state(p, x, k, e, -1.0), oracle_lib.initial_state(p, x, k, e, -1.0)
        assert np.allclose(u1, u2, rtol=1e-13, atol=0)
        x1, k1 = cc.back_transform(p, u2, e)
        assert np.allclose(x1, x, rtol=1e-12, atol=1e-12)                 # round trip position
        pb = oracle_lib.make_params(B0=1e14 * b0sign, **CONFIGS[cfg])
        p1 = cc.prob_single(pb, x, k, e)
        p2 = oracle_lib.get_prob_nonad(pb, x, k, [e])[0]
        assert abs(p1 - p2) <= 1e-9 * abs(p2), (i, p1, p2)


def test_sampler_condition(oracle_lib):
    for cfg in CONFIGS:
        p = oracle_lib.make_params(**CONFIGS[cfg])
        rng = np.random.default_rng(4)
        for _ in range(300):
            x = rng.normal(size=3) * 30
            vl = rng.normal(size=3)
            vl /= np.linalg.norm(vl)
            a, b = cc.sampler_condition(p, x, vl, ERG), oracle_lib.sampler_condition(p, x, vl, ERG)
            assert np.isnan(a) == np.isnan(b)
            if not np.isnan(b):
                assert abs(a - b) <= 1e-10 * (abs(b) + 1e-3)


@pytest.mark.parametrize("kw", [dict(theta_m=0.2, mass_a=1e-5), dict(theta_m=0.0, mass_a=1e-6, B0=2e14),
                                dict(theta_m=1.2, mass_a=3e-6, B0=5e13, omega_pul=2.0),
                                dict(theta_m=0.5, mass_a=1e-5, isotropic=True), dict(theta_m=0.3, mass_a=1e-5, rNS=12.0)])
def test_sampler_sign_fast(kw, oracle_lib):
    """sampler_sign_fast (the sampler grid's signs without the condition) never disagrees with the
    condition where it decides: on the 0.5 km grid of sampler-like lines through the conversion
    region and at points 1e-12..1e-3 km on either side of the grid's sign changes (bisected to
    the root), against the product's condition and, on a subset, the oracle's."""
    p = oracle_lib.make_params(**kw)
    rng = np.random.default_rng(11)
    maxR = 1.2 * (2.0 * (4.0 * np.pi * abs(2.0 * kw.get("omega_pul", 1.0) / np.sqrt(4.0 * np.pi / 137.0) * 1.95e-2
                                            * 6.582119e-16) / 137.0 / 5.0e5 * 0.5 * kw.get("B0", 1e14)
                         * kw.get("rNS", 10.0) ** 3) / kw["mass_a"] ** 2) ** (1.0 / 3.0)
    n = 300
    va = rng.normal(size=(n, 3)); va /= np.linalg.norm(va, axis=1, keepdims=True)
    vl = rng.normal(size=(n, 3)); vl /= np.linalg.norm(vl, axis=1, keepdims=True)
    off = rng.normal(size=(n, 3)); off -= (off * va).sum(1, keepdims=True) * va
    off *= (np.sqrt(rng.random(n)) * maxR / np.linalg.norm(off, axis=1))[:, None]
    x0 = off - 1.1 * maxR * va
    E = 1.0000002692622573 * kw["mass_a"] * (1.0 + 1e-8 * rng.random(n))
    s = np.arange(1, int(2.2 * maxR / 0.5) * 19 + 1) * (0.5 / 19)
    xs = (x0[:, None, :] + va[:, None, :] * s[None, :, None]).reshape(-1, 3)
    c, g = cc.sampler_signs(p, xs, np.repeat(vl, len(s), 0), np.repeat(E, len(s)))
    r = np.linalg.norm(xs, axis=1)
    assert (((g == 1) & ~(c < 0)) | ((g == 2) & ~(c > 0))).sum() == 0
    ext = r > max(10.0, kw.get("rNS", 10.0)) * (1 + 1e-8)
    assert (g[ext] != 0).mean() > 0.999  # decided almost everywhere outside the star
    assert (g[~ext] == 0).all()
    c2 = c.reshape(n, -1)
    i, k = np.nonzero(np.signbit(c2[:, 1:]) != np.signbit(c2[:, :-1]))
    assert len(i) > 20
    sa, sb = s[k].copy(), s[k + 1].copy()

    def f(ss):
        return cc.sampler_signs(p, x0[i] + va[i] * ss[:, None], vl[i], E[i])
    fa = f(sa)[0]
    for _ in range(70):
        sm = 0.5 * (sa + sb)
        fm = f(sm)[0]
        same = np.signbit(fm) == np.signbit(fa)
        sa, fa, sb = np.where(same, sm, sa), np.where(same, fm, fa), np.where(same, sb, sm)
    decided = 0
    for lg in np.arange(-12.0, -2.5, 0.5):
        for sg in (-1.0, 1.0):
            ss = sa + sg * 10.0 ** lg
            cn, gn = f(ss)
            assert (((gn == 1) & ~(cn < 0)) | ((gn == 2) & ~(cn > 0))).sum() == 0
            decided += int((gn != 0).sum())
            if lg in (-8.0, -6.0):
                xo = x0[i] + va[i] * ss[:, None]
                for q in range(0, len(gn), max(1, len(gn) // 40)):
                    if gn[q] != 0:
                        o = oracle_lib.sampler_condition(p, xo[q], vl[i][q], E[i][q])
                        assert (o < 0) if gn[q] == 1 else (o > 0)
    assert decided > 0


def test_metric_derivatives_finite_difference():
    rs = 2.9532
    for r in [9.0, 9.99, 10.0, 10.01, 12.0, 50.0]:
        g = cc.metric_d(r, rs)
        h = 1e-6 * r
        gp, gm = cc.metric_d(r + h, rs), cc.metric_d(r - h, rs)
        if abs(r - 10.0) > 2 * h:  # the interior patch switches at r = 10 (RayTracer.jl:455)
            assert abs((gp[0] - gm[0]) / (2 * h) - g[2]) < 1e-7 * abs(g[2]) + 1e-12
            assert abs((gp[1] - gm[1]) / (2 * h) - g[3]) < 1e-7 * abs(g[3]) + 1e-12
    # the interior and exterior metric meet continuously at r = 10
    a, b = cc.metric_d(10.0, rs), cc.metric_d(np.nextafter(10.0, 11.0), rs)
    assert abs(a[0] - b[0]) < 1e-12 and abs(a[1] - b[1]) < 1e-12
