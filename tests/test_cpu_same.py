"""The same-algorithm CPU baseline (tools/cpu_same.cpp, bench.py's cpu_baseline) runs the
engine's algorithm: it agrees with the oracle on the same seeded rays as closely as the HIP
engine does (statuses, end states, crossings, P), so its timing is a like-for-like figure."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

from conftest import CONFIGS  # noqa: E402


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_same_algorithm_port_matches_oracle(cfg, oracle_lib):
    import cpu_same
    p = oracle_lib.make_params(**CONFIGS[cfg])
    n = 2000
    s = oracle_lib.sample(p, oracle_lib.find_conversion_surface(p), 1769, 0, n)
    o = oracle_lib.propagate(p, s["x"], s["k_init"], s["erg"], -1.0, -30.0, 1)
    c = cpu_same.propagate(p, s["x"], s["k_init"], s["erg"], nthreads=os.cpu_count() or 1)
    same = o["status"] == c["status"]
    assert same.mean() >= 0.99
    rel = np.abs(o["x_end"].reshape(3, n) - c["x_end"].reshape(3, n)).max(0) / np.linalg.norm(
        o["x_end"].reshape(3, n), axis=0)
    assert np.median(rel[same]) < 1e-9 and np.mean(rel[same] > 1e-3) < 0.01
    cr = same & (o["status"] == 1)
    pr = np.abs(o["xc_p"][cr] - c["xc_p"][cr]) / np.abs(o["xc_p"][cr])
    assert np.median(pr) < 1e-9
    assert np.median(np.abs(o["n_accept"][same] - c["n_accept"][same])) == 0
