"""The Vern6 tableau (OrdinaryDiffEq's Vern6, RayTracer.jl:383) is restated from memory of
Verner's published 'most efficient' 6(5) pair; these order conditions pin it: b must satisfy
all 37 conditions of order <= 6 (and fail order 7), bhat all 17 of order <= 5 (and fail 6).
Both the oracle's copy and the kernel's copy (libart.so, no GPU needed) are checked."""
import functools

import numpy as np
import pytest


def trees(n):
    if n == 1:
        return [()]
    out = set()

    def parts(m, maxsz):
        if m == 0:
            yield []
            return
        for s in range(min(m, maxsz), 0, -1):
            for t in trees(s):
                for rest in parts(m - s, s):
                    yield [t] + rest
    for p in parts(n - 1, n - 1):
        out.add(tuple(sorted(p)))
    return list(out)


@functools.lru_cache(None)
def order(t):
    return 1 + sum(order(s) for s in t)


@functools.lru_cache(None)
def gamma(t):
    g = order(t)
    for s in t:
        g *= gamma(s)
    return g


def residual(A, w, t):
    def phi(t):
        v = np.ones(A.shape[0])
        for s in t:
            v = v * (A @ phi(s))
        return v
    return w @ phi(t) - 1.0 / gamma(t)


def check(c, A, b, bh):
    assert np.abs(A.sum(1) - c).max() < 1e-12                     # row-sum (consistency) conditions
    assert np.allclose(A[8], b, rtol=0, atol=0)                    # FSAL: b is the last row
    assert sum(len(trees(o)) for o in range(1, 7)) == 37
    assert max(abs(residual(A, b, t)) for o in range(1, 7) for t in trees(o)) < 1e-10
    assert max(abs(residual(A, bh, t)) for o in range(1, 6) for t in trees(o)) < 1e-11
    assert max(abs(residual(A, b, t)) for t in trees(7)) > 1e-8     # genuinely 6th order
    assert max(abs(residual(A, bh, t)) for t in trees(6)) > 1e-4    # genuinely 5th order


def test_oracle_tableau(oracle_lib):
    check(*oracle_lib.vern6_tableau())


def test_kernel_tableau_identical_to_oracle(oracle_lib):
    from adiabatic_raytracer_amd import vern6_tableau
    k = vern6_tableau()
    o = oracle_lib.vern6_tableau()
    check(*k)
    for a, b in zip(k, o):
        assert np.array_equal(a, b)
