"""The parameter scan (BASELINE.json configs[4], adiabatic_raytracer_amd/scan.py) on the GPU:
two grid points at a small ray count give complete, well-formed records; the flux of a
point equals a direct Engine run of the same point (the scan adds no state of its own)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_scan_points_run():
    import torch
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    from adiabatic_raytracer_amd.scan import run_point, run_scan, scan_grid
    recs = run_scan(2000, n_points=3)  # three points on 4 streams (run_points)
    assert [r["point"] for r in recs] == [0, 1, 2]
    for r in recs:
        assert r["accepted"] > 0 and sum(r["status_counts"]) == 2000 and len(r["flux_photon"]) == 50
    kw = scan_grid()[1]
    eng = Engine(A.Params(**kw))
    inp = eng.forward_roots(2000, seed=1769)
    out = eng.propagate(inp, max_crossings=-1)
    h = eng.flux_histogram(out, inp["species"], None, 50)
    torch.cuda.synchronize()
    assert np.array_equal(h[50:].cpu().numpy(), np.asarray(recs[1]["flux_photon"]))
    # the point-by-point path gives the same records
    seq = run_scan(2000, n_points=3, run=run_point)
    for a, b in zip(recs, seq):
        assert a["accepted"] == b["accepted"] and a["status_counts"] == b["status_counts"]
        assert a["flux_photon"] == b["flux_photon"]



def test_run_points_dispatch_order_and_records():
    """More points than streams: every point runs (largest conversion radius first, each next
    point on the first idle stream), the records come back in grid order with their own
    kernel times, and each equals the point run alone."""
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd.scan import run_point, run_points, scan_grid
    kws = [scan_grid()[i] for i in (24, 6, 17, 1, 30)]
    recs, summ = run_points(kws, 1500, streams=2)
    maxr = [A.Params(**kw).max_r() for kw in kws]
    assert summ["order"] == sorted(range(len(kws)), key=lambda i: -maxr[i])
    assert summ["points"] == len(kws) and summ["accepted"] == sum(r["accepted"] for r in recs)
    for kw, r in zip(kws, recs):
        assert r["mass_a"] == kw["mass_a"] and r["B0"] == kw["B0"] and r["kernel_ms"] > 0
        alone = run_point(kw, 1500, 1769)
        assert r["accepted"] == alone["accepted"] and r["status_counts"] == alone["status_counts"]
        assert r["flux_photon"] == alone["flux_photon"]
