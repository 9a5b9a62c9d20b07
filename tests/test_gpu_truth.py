"""The HIP engine against the converged-truth fixtures (tests/golden/truth_*.npz): final
positions, crossings (x, k, t, Δω), conversion probabilities and the binned flux of the
forward segment (RT.propagate, RayTracer.jl:171-452; get_Prob_nonAD, MainRunner.jl:67-124;
plot/flux.py:38-48) within the north_star's stated FP64 tolerance (tests/truth_compare.py),
through the C ABI (art_propagate_host_flux: the flux is the device histogram).

Missed and extra crossings of the engine's cubic-Hermite scan against the truth's 50-point
scan of the converged dense output are counted and bounded; each comparison is printed as
one JSON line (and appended to $ART_TRUTH_REPORT when set)."""
import json
import os

import numpy as np
import pytest

import truth_compare as T

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["reference", "tight"])
@pytest.mark.parametrize("case", T.CASES)
def test_engine_within_stated_tolerance(case, mode):
    import adiabatic_raytracer_amd as A
    z = T.load(case)
    n = z["n"]
    p = A.Params(**T.NUMERICS[mode], **z["params"])
    g = A.propagate_batch(p, z["x0"], z["k0"], z["erg"], -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8),
                          max_crossings=-1, flux_nbins=50)
    rep = T.compare(z, g)
    rep.update(case=case, mode=mode)
    line = json.dumps(rep)
    print(line)
    if os.environ.get("ART_TRUTH_REPORT"):
        with open(os.environ["ART_TRUTH_REPORT"], "a") as fh:
            fh.write(line + "\n")
    # the device histogram (art_propagate_host_flux) is the engine's own per-ray outputs binned
    # as plot/flux.py:38-48 does, bin for bin; photons only
    assert np.all(g["flux"][0] == 0.0)
    assert np.array_equal(g["flux"][1], T.flux_of(g["status"], g["x_end"], g["k_end"], p.rNS))
    T.check(rep, mode)


@pytest.mark.parametrize("mode", ["reference", "tight"])
@pytest.mark.parametrize("case", ("flat", "gr"))
def test_saved_points_within_stated_tolerance(case, mode):
    """saveat (RayTracer.jl:176,383,427-444, art_propagate_traj_*): the interior saved positions of
    the truth rays that reach ln t_end against the converged dense output at the same times
    (tests/golden/truth_saveat_*.npz), within truth_compare.SAVED_TOL."""
    import adiabatic_raytracer_amd as A
    z, zs = T.load(case), T.load_saved(case)
    n = z["n"]
    p = A.Params(**T.NUMERICS[mode], **z["params"])
    g = A.propagate_batch(p, z["x0"], z["k0"], z["erg"], -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8),
                          max_crossings=-1, ntimes=int(zs["ntimes"]))
    rep = T.compare_saved(zs, g, n)
    rep.update(case=case, mode=mode, what="saved points")
    line = json.dumps(rep)
    print(line)
    if os.environ.get("ART_TRUTH_REPORT"):
        with open(os.environ["ART_TRUTH_REPORT"], "a") as fh:
            fh.write(line + "\n")
    assert rep["compared"]["rays"] >= 0.95 * rep["compared"]["fixture rays"]
    T.check_saved(rep, mode)
