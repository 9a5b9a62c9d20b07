"""Tail donation (art_set_tail_donation, include/art.h) is an execution policy only: a drained
wave hands its last live rays, between steps, to a continuation launch that resumes them from
their complete saved state. Every output and every launch counter must equal the undonated
run bit for bit, for the flat and GR instantiations and for a lane count that donates almost
every wave."""
import numpy as np
import pytest

from conftest import CONFIGS

pytestmark = pytest.mark.gpu

N = 8000


def _run(eng, inp, lanes):
    import torch
    import adiabatic_raytracer_amd as A
    eng.set_tail_donation(lanes)
    torch.cuda.synchronize()
    try:
        # (a non-blocking stream: early graduation, SegOut::hot, runs only on one)
        with torch.cuda.stream(torch.cuda.Stream()):
            out = eng.propagate(inp, max_crossings=-1)
            eng.kernel_ms()
            st = dict(A.raytracer.last_stats())
    finally:
        eng.set_tail_donation(-1)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items() if hasattr(v, "cpu")}, st


@pytest.mark.parametrize("cfg", ["flat", "gr", "gr_oblique"])
@pytest.mark.parametrize("tail", ["0", "100000"], ids=["packed", "tail_kernel"])
def test_tail_donation_is_bit_exact(cfg, tail, monkeypatch):
    """ART_TAIL=0: the donated rays resume packed into full waves (the bulk kernel's own
    continuation); ART_TAIL=100000: every donated ray resumes on a wave of its own (tail_kernel,
    which spreads the attempt's independent work over the lanes)."""
    monkeypatch.setenv("ART_TAIL", tail)
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    eng = Engine(A.Params(**CONFIGS[cfg]))
    inp = eng.forward_roots(N, seed=1769)
    ref, sref = _run(eng, inp, 0)
    has = ref["n_cross"] > 0  # crossing slots of rays without a crossing are never written
    for lanes in (16, 63):
        got, sgot = _run(eng, inp, lanes)
        for k in ref:
            a, b = ref[k], got[k]
            if k.startswith("xc_"):
                a, b = a.reshape(-1, N)[:, has], b.reshape(-1, N)[:, has]
            assert np.array_equal(a, b, equal_nan=True), (cfg, lanes, k)
        for k in ("attempts", "accepted", "root_steps", "scan_evals", "rays", "cert_steps"):
            assert sref[k] == sgot[k], (cfg, lanes, k, sref[k], sgot[k])


@pytest.mark.parametrize("cfg", ["flat", "gr", "gr_oblique"])
@pytest.mark.parametrize("graduate", ["1", "64", "2048"])
def test_graduation_is_bit_exact(cfg, graduate, monkeypatch):
    """ART_GRADUATE=k: a ray still stepping after k attempts leaves its wave for a wave of its own
    (tail_kernel) without waiting for the wave to drain. k=1 graduates nearly every ray (and
    overflows the graduation records, so the rest stay in place), k=64 a large share, 2048 (the
    default) the outliers. Outputs and counters equal the undonated run bit for bit."""
    monkeypatch.setenv("ART_GRADUATE", graduate)
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    eng = Engine(A.Params(**CONFIGS[cfg]))
    inp = eng.forward_roots(N, seed=1769)
    ref, sref = _run(eng, inp, 0)
    has = ref["n_cross"] > 0
    got, sgot = _run(eng, inp, 16)
    for k in ref:
        a, b = ref[k], got[k]
        if k.startswith("xc_"):
            a, b = a.reshape(-1, N)[:, has], b.reshape(-1, N)[:, has]
        assert np.array_equal(a, b, equal_nan=True), (cfg, graduate, k)
    for k in ("attempts", "accepted", "root_steps", "scan_evals", "rays", "cert_steps"):
        assert sref[k] == sgot[k], (cfg, graduate, k, sref[k], sgot[k])


@pytest.mark.parametrize("cfg", ["flat", "gr", "gr_oblique"])
@pytest.mark.parametrize("hot", [("16", "1e9"), ("64", "14"), ("128", "15.95")], ids=["every_ray", "some", "default"])
def test_early_graduation_is_bit_exact(cfg, hot, monkeypatch):
    """ART_HOT_AT=a, ART_HOT_DTAU=d (SegOut::hot): from a attempts on, a ray whose progress in ln t
    lags d + 0.75 log2(attempts / 256) leaves for the hot records at once, and a tail_kernel
    launch beside the bulk pass resumes it as soon as its record is written. a=16, d=1e9 sends
    every ray alive at 16 attempts (and overflows the 1024 records, so the rest stay in place);
    128/15.95 is the default. Outputs and counters equal the undonated run bit for bit."""
    monkeypatch.setenv("ART_HOT_AT", hot[0])
    monkeypatch.setenv("ART_HOT_DTAU", hot[1])
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    eng = Engine(A.Params(**CONFIGS[cfg]))
    inp = eng.forward_roots(N, seed=1769)
    ref, sref = _run(eng, inp, 0)
    has = ref["n_cross"] > 0
    got, sgot = _run(eng, inp, 16)
    for k in ref:
        a, b = ref[k], got[k]
        if k.startswith("xc_"):
            a, b = a.reshape(-1, N)[:, has], b.reshape(-1, N)[:, has]
        assert np.array_equal(a, b, equal_nan=True), (cfg, hot, k)
    for k in ("attempts", "accepted", "root_steps", "scan_evals", "rays", "cert_steps"):
        assert sref[k] == sgot[k], (cfg, hot, k, sref[k], sgot[k])


def test_early_graduation_default_on_a_large_gr_batch(monkeypatch):
    """The default rule and the claim order on 2*10^5 configs[3] rays (rays long enough to be hot
    by it, as in the 10^6-ray batch): every output and counter equals the launch with both off
    (ART_HOT_AT=0), which claims rays in index order and never graduates early."""
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    n = 200000
    eng = Engine(A.Params(**CONFIGS["gr"]))
    inp = eng.forward_roots(n, seed=1769)
    got, sgot = _run(eng, inp, -1)
    monkeypatch.setenv("ART_HOT_AT", "0")
    ref, sref = _run(eng, inp, -1)
    assert int((ref["n_accept"] + ref["n_reject"]).max()) > 4096  # (the batch has long rays)
    has = ref["n_cross"] > 0
    for k in ref:
        a, b = ref[k], got[k]
        if k.startswith("xc_"):
            a, b = a.reshape(-1, n)[:, has], b.reshape(-1, n)[:, has]
        assert np.array_equal(a, b, equal_nan=True), k
    for k in ("attempts", "accepted", "root_steps", "scan_evals", "rays", "cert_steps"):
        assert sref[k] == sgot[k], (k, sref[k], sgot[k])


def test_tail_donation_rejects_bad_lane_counts():
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    eng = Engine(A.Params(**CONFIGS["flat"]))
    for bad in (-2, 64):
        with pytest.raises(A.ArtError):
            eng.set_tail_donation(bad)


def _host_run(p, args, lanes, **kw):
    import adiabatic_raytracer_amd as A
    lib = A._lib.load()
    A._lib.check(lib.art_set_tail_donation(lanes))
    try:
        return A.propagate_batch(p, *args, **kw)
    finally:
        A._lib.check(lib.art_set_tail_donation(-1))


@pytest.mark.parametrize("cfg", ["flat", "gr"])
@pytest.mark.parametrize("mode", ["backtrace", "saveat"])
@pytest.mark.parametrize("tail", ["0", "100000"], ids=["packed", "tail_kernel"])
def test_tail_donation_round_trips_crossings_and_saved_points(cfg, mode, tail, monkeypatch):
    """The donation record carries the post-event state (condition memory, sign, the
    just-evented flag), the crossing count and the next saveat index. Round trips through it
    with several crossings per ray -- the all-crossings axion backtrace (max_crossings 100000,
    capacity 8, -k and -B0 as MainRunner.jl:581-591) -- and with saved points (ntimes 3 and 7,
    RayTracer.jl:176,383) leave every output bit-identical (host entry points, which honour the
    device's donation setting like every launch)."""
    from dataclasses import replace
    import adiabatic_raytracer_amd as A
    monkeypatch.setenv("ART_TAIL", tail)
    p = A.Params(**CONFIGS[cfg])
    n = 4000
    s = A.sample_conversion_points(p, n, seed=1769)
    if mode == "backtrace":
        q = replace(p, B0=-p.B0)
        args = (s["x"], -s["k_init"], s["erg"], -np.ones(n), np.full(n, -30.0), np.zeros(n, np.int8))
        kws = [dict(max_crossings=100000, capacity=8)]
    else:
        q = p
        args = (s["x"], s["k_init"], s["erg"], -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8))
        kws = [dict(max_crossings=-1, capacity=1, ntimes=3), dict(max_crossings=-1, capacity=1, ntimes=7)]
    for kw in kws:
        ref = _host_run(q, args, 0, **kw)
        if mode == "backtrace":
            assert (ref["n_cross"] > 1).any()
        for lanes in (16, 63):
            got = _host_run(q, args, lanes, **kw)
            for k, v in ref.items():
                if isinstance(v, np.ndarray):
                    assert np.array_equal(v, got[k], equal_nan=True), (cfg, mode, kw, lanes, k)
            for k in ("attempts", "accepted", "root_steps", "scan_evals", "rays", "cert_steps"):
                assert ref["stats"][k] == got["stats"][k], (cfg, mode, lanes, k)
