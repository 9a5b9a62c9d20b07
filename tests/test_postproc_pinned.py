"""The build's radiated flux and event_/final_ text files against the reference's own
post-processing scripts, run unchanged on build-written files (tests/golden/make_postproc_fixture.py).

tests/golden/flux_py/: what plot/flux.py computed from results/combined.npy = the reference's
Combine_Files.py output over two build-written 29-column row files (tests/golden/combine_py/):
the (hist, bin_edges) of its np.histogram calls -- flux.py:43-47 first, the photon and then the
axion flux over 50 data-dependent bins -- and its printed tree statistics.

tests/golden/analysis_py/: event_/final_ text files the GPU build wrote (saveMode 2,
MainRunner.jl:592-609, 690-702) and the columns jonas_test_analyses/analysis.py's own
load_event_info / load_final_info (:8-33) returned for them, plus its np.histogram calls
(the differential power over θf, :91-96)."""
import os

import numpy as np
import pytest

G = os.path.join(os.path.dirname(__file__), "golden")
FLUX = os.path.join(G, "flux_py", "flux_calls.npz")
ANA = os.path.join(G, "analysis_py", "analysis_calls.npz")
TAG = "convergence_1e-10"
EVENT_COLS = ("num", "vIfty", "sln_prob", "x_in", "k_in", "x0", "k0", "time", "nodes")
FINAL_COLS = ("num", "weight", "species", "theta_f", "phi_f", "abs_f", "theta_Xf", "phi_Xf", "abs_Xf", "t")


def _rows():
    return np.load(os.path.join(G, "combine_py", "expected_mode1.npy"))


@pytest.mark.skipif(not os.path.exists(FLUX), reason="fixture not generated")
def test_flux_py_bins_are_the_builds():
    """flux.py bins φf (column 4) over [min, max] of ALL rows (np.histogram without a range);
    trees.flux_range / flux_edges give exactly those edges, and the recorded photon / axion
    histograms are the flux of weight * sln_prob (columns 9 and 8) by particle id (column 2)."""
    from adiabatic_raytracer_amd.trees import flux_edges, flux_range
    z = np.load(FLUX)
    assert str(z["error"]) == "", z["error"]  # flux.py ran to its end on the build's 29-column rows
    rows = _rows()
    phif, pid, pps = rows[:, 3], rows[:, 1], rows[:, 8] * rows[:, 7]
    lo, hi = flux_range(phif)
    for k in (0, 1):
        assert np.array_equal(z[f"edges{k}"], flux_edges(lo, hi, 50))
    assert z["hist0"].shape == (50,) and z["hist1"].shape == (50,)
    # the photon and axion totals: every row falls in [lo, hi]
    assert np.isclose(z["hist0"].sum(), pps[pid == 1].sum(), rtol=1e-13)
    assert np.isclose(z["hist1"].sum(), pps[pid == 0].sum(), rtol=1e-13)


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(FLUX), reason="fixture not generated")
def test_device_flux_equals_flux_py():
    """The product's radiated flux (trees.radiated_flux: flux_phi_kernel on the GPU) over the
    same rows and flux.py's data-dependent bins equals what the reference's flux.py computed, bin
    for bin (to the rounding of a differently ordered weighted sum)."""
    import adiabatic_raytracer_amd as A
    z = np.load(FLUX)
    rows = _rows()
    h = A.trees.radiated_flux(rows[:, 3], rows[:, 1], rows[:, 8] * rows[:, 7], 50, range=None).reshape(2, 50)
    np.testing.assert_allclose(h[1], z["hist0"], rtol=1e-12, atol=0)  # photons (flux.py:43-44)
    np.testing.assert_allclose(h[0], z["hist1"], rtol=1e-12, atol=0)  # axions (flux.py:46-47)
    # and the fixed [-π, π] binning the run totals use is the same histogram over those edges
    hp = A.trees.radiated_flux(rows[:, 3], rows[:, 1], rows[:, 8] * rows[:, 7], 50).reshape(2, 50)
    ref = np.histogram(rows[:, 3], 50, range=(-np.pi, np.pi), weights=rows[:, 8] * rows[:, 7] * (rows[:, 1] == 1))[0]
    np.testing.assert_allclose(hp[1], ref, rtol=1e-12, atol=0)


def _parse_event(path):
    """The build's own reading of its event_ file (MainRunner.jl:592-609): event number, vIfty
    (3), sln_prob, x_in (3), k_in (3), x0 (3), k0 (3), time, nodes."""
    d = np.loadtxt(path, ndmin=2)
    return {"num": d[:, 0], "vIfty": d[:, 1:4], "sln_prob": d[:, 4], "x_in": d[:, 5:8], "k_in": d[:, 8:11],
            "x0": d[:, 11:14], "k0": d[:, 14:17], "time": d[:, 17], "nodes": d[:, 18]}


def _parse_final(path):
    """... and of its final_ file (MainRunner.jl:690-702): event number, weight, species, θf, φf,
    |k|, θXf, φXf, |x|, t."""
    d = np.loadtxt(path, ndmin=2)
    return dict(zip(FINAL_COLS, (d[:, 0].astype(int), *(d[:, c] for c in range(1, 10)))))


@pytest.mark.skipif(not os.path.exists(ANA), reason="fixture not generated")
def test_event_final_layout_as_analysis_py_reads_it():
    """What analysis.py's loaders returned for the build's files is what the build means by its
    columns: the event numbers, vIfty, sln_prob, the forward and backward start momenta and the
    node counts of event_, and every column of final_ (the reference's loader slices event_'s
    x_in/k_in as 4-column blocks, x_in = columns 5-8: its indices are kept as they are)."""
    z = np.load(ANA)
    ev = _parse_event(os.path.join(G, "analysis_py", "event_" + TAG))
    fi = _parse_final(os.path.join(G, "analysis_py", "final_" + TAG))
    assert np.array_equal(z["event_num"], ev["num"])
    assert np.array_equal(z["event_vIfty"], ev["vIfty"])
    assert np.array_equal(z["event_sln_prob"], ev["sln_prob"])
    assert np.array_equal(z["event_time"], ev["time"]) and np.array_equal(z["event_nodes"], ev["nodes"])
    raw = np.loadtxt(os.path.join(G, "analysis_py", "event_" + TAG), ndmin=2)
    assert np.array_equal(z["event_x_in"], raw[:, 5:9]) and np.array_equal(z["event_k0"], raw[:, 17:-2])
    for c in FINAL_COLS:
        assert np.array_equal(z["final_" + c], fi[c]), c
    # events are numbered 1..N in event_, every final_ row belongs to one of them (analysis.py:87
    # indexes event rows by num - 1), species is 0/1
    assert np.array_equal(ev["num"], np.arange(1, len(ev["num"]) + 1))
    assert fi["num"].min() >= 1 and fi["num"].max() <= len(ev["num"])
    assert set(np.unique(fi["species"])) <= {0.0, 1.0}
    assert str(z["error"]) == ""


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(ANA), reason="fixture not generated")
def test_regenerated_event_files_match_fixture(tmp_path):
    """The GPU build, run again with the fixture's parameters, writes the same event_/final_
    files: the same events, trees and species, the same values to 1e-9 (the per-event wall
    time column excepted), so analysis.py reads the current build's files as it read the
    fixture's."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("mk", os.path.join(G, "make_postproc_fixture.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    mk.stage_gpu(str(tmp_path))
    d = os.path.join(str(tmp_path), "results", "event")
    ev_new, fi_new = _parse_event(os.path.join(d, "event_" + TAG)), _parse_final(os.path.join(d, "final_" + TAG))
    ev_fix = _parse_event(os.path.join(G, "analysis_py", "event_" + TAG))
    fi_fix = _parse_final(os.path.join(G, "analysis_py", "final_" + TAG))
    for c in EVENT_COLS:
        if c != "time":  # (wall time per event)
            np.testing.assert_allclose(ev_new[c], ev_fix[c], rtol=1e-9, atol=1e-12, err_msg=c)
    assert np.array_equal(fi_new["num"], fi_fix["num"]) and np.array_equal(fi_new["species"], fi_fix["species"])
    for c in FINAL_COLS[1:]:
        np.testing.assert_allclose(fi_new[c], fi_fix[c], rtol=1e-9, atol=1e-12, err_msg=c)
