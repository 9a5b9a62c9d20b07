"""Philox4x32-10 known-answer vectors (Random123 kat_vectors), for the oracle and for the
kernel header's implementation (host build). The RNG replaces Julia's global stream
(SURVEY §7 hard part iv), so initial conditions depend only on (seed, ray id)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

KATS = [
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


@pytest.mark.parametrize("ctr,key,expect", KATS)
def test_oracle_philox_kat(oracle_lib, ctr, key, expect):
    assert oracle_lib.philox4x32_10(ctr, key) == expect


@pytest.mark.parametrize("ctr,key,expect", KATS)
def test_kernel_philox_kat(ctr, key, expect):
    import corecheck
    assert corecheck.philox(ctr, key) == expect


def test_attempt_uniforms_identical(oracle_lib):
    import corecheck
    for seed, ray, att in [(1769, 0, 0), (1769, 12345678901, 7), (2**40 + 3, 2**33, 2**31)]:
        u1 = np.zeros(10)
        import ctypes as C
        oracle_lib.lib().oracle_attempt_uniforms(seed, ray, att, u1.ctypes.data_as(C.POINTER(C.c_double)))
        u2 = corecheck.attempt_uniforms(seed, ray, att)
        assert np.array_equal(u1, u2)
        assert np.all((u1 >= 0) & (u1 < 1))
