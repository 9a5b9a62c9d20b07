"""Asynchronous host calls (art_propagate_host_flux_async / art_host_wait, include/art.h).

MainRunner.jl:179-190 hands RT.propagate one batch after another; a host that has the next batch
ready submits it before waiting for this one, so its uploads and first rays overlap this batch's
drain. Two calls per device are in flight, each on its own host lane (streams, staging, host
words). On the GPU (`-m gpu`):
* calls in flight return exactly the synchronous single launch's outputs -- every crossing slot,
  the flux, the statistics -- for flat and GR photons and all-crossings axion backtraces, with
  three batches chained two deep (submit A, B; wait A; submit C; wait B, C);
* a call whose streamed pipeline gives up inside the worker (piece bound 0 ms) runs again as one
  launch on its lane's stream and staging, with the same outputs; the next async call streams;
* a batch below the streamed pipeline's size runs inside the submitting call (ticket complete);
* tickets are waited for once: an unknown or already waited ticket is ART_E_INVALID;
* a synchronous call after async ones waits for them and uses lane 0 safely.
"""
import numpy as np
import pytest

from conftest import CONFIGS
from test_edges import host_flux


def _batch(A, p, n, species, seed_offset=0):
    from dataclasses import replace
    s = A.sample_conversion_points(p, n + seed_offset, seed=1769)
    x, k = s["x"].reshape(3, -1)[:, seed_offset:].ravel(), s["k_init"].reshape(3, -1)[:, seed_offset:].ravel()
    erg = s["erg"][seed_offset:]
    if species == 0:  # the backtrace (MainRunner.jl:581-591): axions, -B0, -k, all crossings
        return replace(p, B0=-p.B0), (x, -k, erg, -np.ones(n), np.full(n, -30.0), np.zeros(n, np.int8)), 100000
    return p, (x, k, erg, -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8)), -1


def _same(ref, got, tag):
    for key, v in ref.items():
        if isinstance(v, np.ndarray):
            assert np.array_equal(v, got[key], equal_nan=True), (tag, key)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,species,cap", [("flat", 1, 1), ("gr", 1, 2), ("flat", 0, 3)])
def test_async_calls_in_flight_are_bit_exact(cfg, species, cap, monkeypatch):
    import adiabatic_raytracer_amd as A
    p = A.Params(**CONFIGS[cfg])
    sizes = (20011, 15013, 17011)
    batches = [_batch(A, p, m, species, seed_offset=o) for m, o in zip(sizes, (0, 20011, 35024))]
    monkeypatch.setenv("ART_HOST_MODE", "single")
    refs = [A.propagate_batch(q, *args, max_crossings=mc, capacity=cap, flux_nbins=50) for q, args, mc in batches]
    monkeypatch.setenv("ART_HOST_MODE", "stream")
    monkeypatch.setenv("ART_HOST_PIECE_SHIFT", "11")
    monkeypatch.setenv("ART_HOST_CHUNK_MIN", "1000")
    A.raytracer.host_path_counters(reset=True)
    sub = lambda i: A.raytracer.propagate_batch_async(batches[i][0], *batches[i][1], flux_nbins=50,  # noqa: E731
                                                      max_crossings=batches[i][2], capacity=cap)
    ha, hb = sub(0), sub(1)
    got_a = ha.wait()
    hc = sub(2)
    got_b, got_c = hb.wait(), hc.wait()
    for i, got in enumerate((got_a, got_b, got_c)):
        _same(refs[i], got, (cfg, i))
        assert np.array_equal(got["flux"], refs[i]["flux"]), (cfg, i)
        assert np.array_equal(got["flux"], host_flux(batches[i][0], got, batches[i][1][5], 50)), (cfg, i)
    assert A.raytracer.host_path_counters() == {"calls": 3, "streamed": 3, "stream_giveups": 0, "chunked": 0,
                                                "single": 0}
    # a synchronous call afterwards (lane 0 again) agrees too, and its statistics are the single launch's
    got = A.propagate_batch(batches[0][0], *batches[0][1], max_crossings=batches[0][2], capacity=cap, flux_nbins=50)
    _same(refs[0], got, (cfg, "sync after async"))
    for key in ("attempts", "accepted", "root_steps", "scan_evals", "rays", "init_rhs", "cert_steps"):
        assert refs[0]["stats"][key] == got["stats"][key], key


@pytest.mark.gpu
def test_async_give_up_runs_again_on_the_lane(monkeypatch):
    import adiabatic_raytracer_amd as A
    p = A.Params(**CONFIGS["flat"])
    q, args, mc = _batch(A, p, 20011, 1)
    monkeypatch.setenv("ART_HOST_MODE", "single")
    ref = A.propagate_batch(q, *args, flux_nbins=50)
    monkeypatch.setenv("ART_HOST_MODE", "stream")
    monkeypatch.setenv("ART_HOST_PIECE_SHIFT", "11")
    monkeypatch.setenv("ART_HOST_CHUNK_MIN", "1000")
    A.raytracer.host_path_counters(reset=True)
    monkeypatch.setenv("ART_HOST_STREAM_TIMEOUT_MS", "0")
    h1 = A.raytracer.propagate_batch_async(q, *args, flux_nbins=50)
    got = h1.wait()
    _same(ref, got, "give-up")
    assert np.array_equal(got["flux"], ref["flux"])
    monkeypatch.setenv("ART_HOST_STREAM_TIMEOUT_MS", "30000")
    got = A.raytracer.propagate_batch_async(q, *args, flux_nbins=50).wait()
    _same(ref, got, "after give-up")
    assert A.raytracer.host_path_counters() == {"calls": 2, "streamed": 1, "stream_giveups": 1, "chunked": 0,
                                                "single": 1}


@pytest.mark.gpu
def test_async_small_batch_and_tickets():
    import ctypes as C
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd._lib import ArtError
    p = A.Params(**CONFIGS["flat"])
    q, args, mc = _batch(A, p, 300, 1)
    ref = A.propagate_batch(q, *args, flux_nbins=50)
    h = A.raytracer.propagate_batch_async(q, *args, flux_nbins=50)  # below the streamed size: runs at submit
    _same(ref, h.wait(), "small")
    lib = A._lib.load()
    with pytest.raises(ArtError):
        A._lib.check(lib.art_host_wait(h.ticket))  # waited for already
    with pytest.raises(ArtError):
        A._lib.check(lib.art_host_wait(C.c_int64(1 << 40)))
    # a bad argument fails at submit, with no ticket
    with pytest.raises(ArtError):
        A.raytracer.propagate_batch_async(q, *args, flux_nbins=0)
