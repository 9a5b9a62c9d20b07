"""The oracle against the converged-truth fixtures (tests/golden/truth_*.npz): the stated FP64
tolerance of the physics outputs (tests/truth_compare.py) holds for the restated reference
algorithm at the reference's tolerances, and the restatement converges to the truth as the
tolerances tighten. The same bounds are applied to the HIP engine in test_gpu_truth.py."""
import os
import sys

import numpy as np
import pytest

import truth_compare as T

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("mode", ["reference", "tight"])
@pytest.mark.parametrize("case", T.CASES)
def test_oracle_within_stated_tolerance(case, mode, oracle_lib):
    z = T.load(case)
    p = oracle_lib.make_params(**T.NUMERICS[mode], **z["params"])
    o = oracle_lib.propagate(p, z["x0"], z["k0"], z["erg"], -1.0, -30.0, 1, max_crossings=-1)
    rep = T.compare(z, o)
    T.check(rep, mode)
    assert rep["compared"]["crossings"] >= 256 and rep["truth_singular"] <= 0.03 * rep["rays"]


def test_tolerance_is_the_solver_not_the_scan(oracle_lib):
    """Every p90 error falls by >= 30x from reltol 1e-7 to 1e-9 (Vern6's error scales with its
    tolerance): the errors the stated tolerance allows are the integrator's, not the scan's."""
    z = T.load("gr_oblique")
    errs = {}
    for rt in (1e-7, 1e-9):
        p = oracle_lib.make_params(abstol=10 * rt, reltol=rt, **z["params"])
        o = oracle_lib.propagate(p, z["x0"], z["k0"], z["erg"], -1.0, -30.0, 1)
        errs[rt] = T.compare(z, o)["errors"]
    for what in ("crossing position", "crossing t", "P_nonAD", "end position"):
        assert errs[1e-9][what][1] * 30 <= errs[1e-7][what][1], (what, errs[1e-7][what], errs[1e-9][what])


@pytest.mark.parametrize("case", T.CASES)
def test_truth_fixture_reproduced(case, oracle_lib):
    """The committed truth is what make_truth_fixture.py computes now (8 rays per case)."""
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_truth_fixture as M
    z = T.load(case)
    n = z["n"]
    x0, k0 = z["x0"].reshape(3, n), z["k0"].reshape(3, n)
    for i in np.linspace(0, n - 1, 8).astype(int):
        r = M.truth_ray((z["params"], x0[:, i].copy(), k0[:, i].copy(), float(z["erg"][i])))
        assert r["status"] == z["status"][i]
        if r["status"] == T.ST_CROSSING:
            assert np.allclose(r["xc"], z["xc_pos"].reshape(3, n)[:, i], rtol=1e-10, atol=0)
            assert np.isclose(r["pc"], z["xc_p"][i], rtol=1e-8, atol=0)
        elif r["status"] == T.ST_SUCCESS:
            assert np.allclose(r["x_end"], z["x_end"].reshape(3, n)[:, i], rtol=1e-10, atol=0)


def test_truth_flux_is_the_fixture_histogram():
    for case in T.CASES:
        z = T.load(case)
        f = T.flux_of(z["status"], z["x_end"], z["k_end"], z["params"].get("rNS", 10.0))
        assert np.array_equal(f, z["flux"]) and f.sum() > 0.15 * z["n"]


@pytest.mark.parametrize("case", ("flat", "gr"))
def test_truth_saveat_fixture_reproduced(case, oracle_lib):
    """The committed saved points are what make_truth_saveat_fixture.py computes now (4 rays)."""
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_truth_saveat_fixture as MS
    z, zs = T.load(case), T.load_saved(case)
    n = z["n"]
    x0, k0 = z["x0"].reshape(3, n), z["k0"].reshape(3, n)
    assert np.all(z["status"][zs["rays"]] == T.ST_SUCCESS)
    for j in np.linspace(0, zs["rays"].size - 1, 4).astype(int):
        i = int(zs["rays"][j])
        pts = MS.saved_points((z["params"], x0[:, i].copy(), k0[:, i].copy(), float(z["erg"][i]), zs["times"]))
        assert np.allclose(pts, zs["pos"][:, :, j], rtol=1e-10, atol=0)
