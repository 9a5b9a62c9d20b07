import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs libart.so kernels)")
    config.addinivalue_line("markers", "slow: longer CPU test")


# Reference configurations (BASELINE.json configs / SURVEY §8d)
CONFIGS = {
    # configs[0..2]: flat space, m_a = 1e-5, θm = 0.2
    "flat": dict(theta_m=0.2, mass_a=1e-5, flat=True),
    # configs[3]: Schwarzschild GR, runner_GR_tasks.sh:10-14
    "gr": dict(theta_m=0.0, mass_a=1e-6, flat=False),
    # GR with a rotating oblique dipole (du7 != 0 path)
    "gr_oblique": dict(theta_m=0.2, mass_a=1e-5, flat=False),
}


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle


def random_states(n, seed=0, rmin=10.5, rmax=60.0, erg=1.0000002692622573e-05):
    """Plausible ODE states u = [r θ φ w_r w_θ w_φ u7] (SoA) for pointwise parity."""
    rng = np.random.default_rng(seed)
    r = rng.uniform(rmin, rmax, n)
    th = rng.uniform(0.05, np.pi - 0.05, n)
    ph = rng.uniform(-np.pi, np.pi, n)
    # direction -> covariant components of a unit-ish momentum (w = k/erg)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    wr = d[:, 0] * 1e-3
    wt = d[:, 1] * r * 1e-3
    wp = d[:, 2] * r * np.sin(th) * 1e-3
    u7 = -erg * rng.uniform(0.999999, 1.000001, n)
    tau = rng.uniform(-30.0, -5.0, n)
    return np.stack([r, th, ph, wr, wt, wp, u7]), tau
