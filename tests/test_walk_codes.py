"""The bit-parallel sign walk (walk_codes_bits, art_core.h) leaves exactly the state of the
sequential walk (walk_codes_loop, the ContinuousCallback's scan order) on random code
sequences: mixtures of positive / negative / NaN runs, every start point and remembered
sign, and 49 (interp_points = 50) as well as other grid sizes. With an exact-zero code in
the range it must decline and leave the work to the loop."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import corecheck as cc  # noqa: E402


def _words(codes):
    cw = [0, 0, 0, 0]
    for i, c in enumerate(codes):  # point i + 1
        cw[i >> 4] |= int(c) << (2 * (i & 15))
    return cw


def _runs(rng, nper, p_zero):
    """Codes in runs, the way signs change along a step (plus isolated flips)."""
    out = []
    while len(out) < nper:
        c = rng.choice([1, 2, 3], p=[0.4, 0.4, 0.2])
        out += [c] * int(rng.integers(1, 12))
    out = np.array(out[:nper])
    flips = rng.random(nper) < 0.05
    out[flips] = rng.choice([1, 2, 3], size=flips.sum())
    out[rng.random(nper) < p_zero] = 0
    return out


@pytest.mark.parametrize("nper", [49, 1, 2, 16, 17, 31, 32, 33, 48, 63, 64])
def test_bits_equal_loop(nper):
    rng = np.random.default_rng(nper)
    declined = 0
    for trial in range(600):
        codes = _runs(rng, nper, p_zero=0.01 if trial % 3 == 0 else 0.0)
        cw = _words(codes)
        ip = int(rng.integers(1, nper + 2))
        last_s = int(rng.choice([-1, 0, 1]))
        last_j = int(rng.integers(0, ip))
        st = [ip, last_s, last_j, int(rng.integers(0, 2))]
        fl, sl = cc.walk(cw, nper, st, bits=False)
        fb, sb = cc.walk(cw, nper, st, bits=True)
        if fb == -1:
            declined += 1
            assert np.any(codes[ip - 1:] == 0)
            continue
        assert (fb, sb) == (fl, sl), (nper, codes.tolist(), st)
    assert declined < 600


def test_found_and_not_found_cases():
    # + + - : change at point 3; the remembered sign was + and point 2 the last nonzero
    assert cc.walk(_words([1, 1, 2]), 3, [1, 0, 0, 1], True) == (1, [3, 1, 2, 0])
    # NaN in between resets: + NaN - has no change
    assert cc.walk(_words([1, 3, 2]), 3, [1, 0, 0, 1], True) == (0, [4, -1, 3, 0])
    # change against the remembered sign at the first point
    assert cc.walk(_words([2, 2]), 2, [1, 1, 0, 1], True) == (1, [1, 1, 0, 1])
    # a zero code declines
    assert cc.walk(_words([1, 0, 2]), 3, [1, 0, 0, 1], True)[0] == -1
