"""Soundness of the certified resonance scan (art_core.h scan_certified_code),
on the host build of the product header (tools/corecheck): for random steps
(u0, f(u0)) -> (u1, f(u1)) over h, whenever the certificate returns "negative" the ORACLE's
condition (RayTracer.jl:254-298) is negative -- not NaN, not zero -- at every grid point the
kernel would have scanned (interp_points = 50 on the cubic Hermite interpolant,
RayTracer.jl:358), whenever it returns "positive" it is positive at every point, and
whenever it returns "NaN" the condition is NaN at every grid point -- in the one-sided form
(b at the end point only: a ray's first step) and the two-sided one (b at both ends).
Both must fire on a good share of the steps, and "negative" never where |u7| < m_a or where
the step can reach the conversion surface."""
import os
import sys

import numpy as np
import pytest

from conftest import CONFIGS, random_states

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import corecheck as cc  # noqa: E402

ERG = 1.0000002692622573e-05


def hermite(u0, f0, u1, f1, h, th):
    a, b = 1.0 - th, th * (th - 1.0)
    return a * u0 + th * u1 + b * ((1.0 - 2.0 * th) * (u1 - u0) + (th - 1.0) * h * f0 + th * h * f1)


@pytest.mark.parametrize("two_sided", [False, True])
@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_certificate_is_sound(cfg, two_sided, oracle_lib):
    kw = dict(CONFIGS[cfg])
    p = oracle_lib.make_params(**kw)
    mr = oracle_lib.find_conversion_surface(p)
    erg = kw["mass_a"] * 1.0000002692622573
    rng = np.random.default_rng(7)
    U1, tau1 = random_states(400, seed=11, rmin=10.5, rmax=12 * mr, erg=erg)
    U2, tau2 = random_states(400, seed=12, rmin=10.5, rmax=mr, erg=erg)  # inside the surface
    U, tau = np.concatenate([U1, U2], axis=1), np.concatenate([tau1, tau2])
    th_grid = np.arange(1, 50) / 49.0
    fired = fired_nan = fired_pos = nan_side = fired_more = 0
    for i in range(U.shape[1]):
        u0, t0 = U[:, i], tau[i]
        f0 = oracle_lib.rhs(p, 1, u0, t0, erg)
        h = 10 ** rng.uniform(-4, 0)
        um = u0 + 0.5 * h * f0
        u1 = u0 + h * oracle_lib.rhs(p, 1, um, t0 + 0.5 * h, erg)
        f1 = oracle_lib.rhs(p, 1, u1, t0 + h, erg)
        if not (np.all(np.isfinite(u1)) and np.all(np.isfinite(f1))):
            continue
        code = cc.certified_code(p, u0, f0, u1, f1, h, t0, two_sided)
        if two_sided:  # the two-sided form certifies whatever the one-sided one does, alike
            c1 = cc.certified_code(p, u0, f0, u1, f1, h, t0, False)
            assert c1 == 0 or c1 == code, (i, c1, code)
            fired_more += code != 0 and c1 == 0
        if abs(u0[6]) < kw["mass_a"] or abs(u1[6]) < kw["mass_a"]:
            nan_side += 1
            assert code not in (1, 2)  # a step that reaches |u7| < m_a is never certified signed
        if code == 0:
            continue
        c = np.array([oracle_lib.condition(p, hermite(u0, f0, u1, f1, h, th), t0 + th * h) for th in th_grid])
        if code == 2:
            fired += 1
            assert np.all(c < 0.0), (i, c.max())
        elif code == 1:
            fired_pos += 1
            assert np.all(c > 0.0), (i, c.min())
        else:
            fired_nan += 1
            assert code == 3 and np.all(np.isnan(c)), (i, code, c)
    assert fired >= 100 and fired_pos >= 20, (fired, fired_pos)
    if kw["flat"]:  # in GR, -g^tt > 1 keeps NrmSq > 0 unless u7 drops by ~rs/r
        assert fired_nan >= 20, fired_nan
    assert nan_side > 0
    if two_sided and kw["flat"]:  # (the random GR steps here are too long to gain)
        assert fired_more > 0


def test_certificate_rejects_the_conversion_surface(oracle_lib):
    """A step that starts on the conversion surface (a sampled conversion point in GR, where
    the sampler's metric is the propagation's) is never certified: its condition is ~0
    there. (In flat space the sampler's GR surface lies 0.5-10% inside the flat one, so
    flat-space roots start at a clearly positive condition.)"""
    kw = CONFIGS["gr"]
    p = oracle_lib.make_params(**kw)
    s = oracle_lib.sample(p, oracle_lib.find_conversion_surface(p), 1769, 0, 64)
    n = 64
    for i in range(n):
        x, k = s["x"].reshape(3, n)[:, i], s["k_init"].reshape(3, n)[:, i]
        u0 = oracle_lib.initial_state(p, x, k, s["erg"][i], -1.0)
        f0 = oracle_lib.rhs(p, 1, u0, -30.0, s["erg"][i])
        u1 = u0 + 1e-3 * f0
        f1 = oracle_lib.rhs(p, 1, u1, -30.0 + 1e-3, s["erg"][i])
        assert cc.certified_code(p, u0, f0, u1, f1, 1e-3, -30.0) == 0
