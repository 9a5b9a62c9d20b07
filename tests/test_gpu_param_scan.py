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

