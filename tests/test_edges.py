"""Edge cases of the drop-in boundary and of the batch.

Without a GPU:
* argument validation runs before any device call. Out-of-range sizes and missing buffers
  give ART_E_INVALID with a message. An empty batch (n = 0) is ART_OK and writes nothing.

On the GPU (`-m gpu`):
* a ray's result does not depend on the batch around it. The same rays in ragged batches
  (1, 63, 65, 257 rays) and in a shuffled batch of 1000 give bit-identical outputs. That
  holds for every lane assignment, wave composition and queue order of the persistent
  integrator. Crossing slots a ray does not fill come back as NaN from the host entry point,
  never as stale staging memory.
* a 70000-ray batch and its first 2000 rays as a batch of their own agree bit for bit (the
  small batch runs the 1-wave/SIMD build, the large one the 2-wave build).
* crossing capacity 8 on flat photon and axion batches of 2000 rays (the batch shape whose
  1-wave/SIMD launch round 2 reported as failed) records the same first crossing as
  capacity 1, also as the first propagate launch of a fresh process (the reproducer of that
  report): the runtime's occupancy query fails for that kernel, and its error must not be
  taken for a launch failure.
* crossing-buffer overflow. An all-crossings axion backtrace (MainRunner.jl:588) into
  capacity 1 reports each ray's full count (> capacity, as include/art.h specifies). It
  stores the same first crossing and end state as the same batch with capacity 8.
"""
import ctypes as C

import numpy as np
import pytest

from conftest import CONFIGS


def _bufs(n, cap=1):
    from adiabatic_raytracer_amd._lib import CrossingBuf, SegmentOut
    out = {"x_end": np.full(3 * n, 7.0), "k_end": np.full(3 * n, 7.0), "u7_end": np.full(n, 7.0),
           "tau_end": np.full(n, 7.0), "status": np.full(n, 7, np.int32), "n_accept": np.full(n, 7, np.int32),
           "n_reject": np.full(n, 7, np.int32), "n_cross": np.full(n, 7, np.int32),
           "xc_pos": np.full(3 * cap * n, 7.0), "xc_k": np.full(3 * cap * n, 7.0), "xc_t": np.full(cap * n, 7.0),
           "xc_dw": np.full(cap * n, 7.0), "xc_p": np.full(cap * n, 7.0)}
    P = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    so = SegmentOut(*[P(out[k]) for k in ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept", "n_reject")])
    xb = CrossingBuf(cap, *[P(out[k]) for k in ("n_cross", "xc_pos", "xc_k", "xc_t", "xc_dw", "xc_p")])
    return out, so, xb


def _host_call(n, so, xb, arrays=True):
    import adiabatic_raytracer_amd as A
    lib = A.load_library()
    cp = A.Params(**CONFIGS["flat"]).to_c()
    m = min(max(n, 1), 16)  # out-of-range n must fail before any buffer is read
    x = np.ones(3 * m)
    e = np.ones(m)
    sp = np.ones(m, np.int8)
    P = lambda a: a.ctypes.data_as(C.c_void_p) if arrays else None  # noqa: E731
    return lib, lib.art_propagate_host(C.byref(cp), n, P(x), P(x), P(e), P(e), P(e), P(sp), -1,
                                       C.byref(so), C.byref(xb))


def test_empty_batch_is_ok_and_writes_nothing():
    out, so, xb = _bufs(1)
    lib, rc = _host_call(0, so, xb)
    assert rc == 0
    assert np.all(out["x_end"] == 7.0) and np.all(out["status"] == 7)


@pytest.mark.parametrize("n", [-1, 2**31])
def test_batch_size_out_of_range(n):
    out, so, xb = _bufs(1)
    lib, rc = _host_call(n, so, xb)
    assert rc == -1 and b"n must be" in lib.art_last_error()


def test_missing_buffers_fail_loudly():
    out, so, xb = _bufs(4)
    lib, rc = _host_call(4, so, xb, arrays=False)
    assert rc == -1 and b"non-NULL" in lib.art_last_error()
    so.x_end = None
    lib, rc = _host_call(4, so, xb)
    assert rc == -1 and b"non-NULL" in lib.art_last_error()


# ---------------------------------------------------------------------------------------
KEYS = ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept", "n_reject", "n_cross", "xc_pos", "xc_k", "xc_t",
        "xc_dw", "xc_p")


def host_flux(p, out, species, nbins):
    """The binned radiated flux of plot/flux.py:38-48 over a batch's host outputs, in numpy:
    segments that end without a crossing beyond 1.1 rNS (MainRunner.jl:203-209), binned by
    atan2(k_y, k_x) over [-pi, pi], axions in row 0 and photons in row 1."""
    n = species.size
    x, k = out["x_end"].reshape(3, n), out["k_end"].reshape(3, n)
    fin = (out["status"] != 1) & (np.sqrt((x * x).sum(0)) > 1.1 * p.rNS)
    phi = np.arctan2(k[1], k[0])
    return np.stack([np.histogram(phi[fin & (species == s)], nbins, range=(-np.pi, np.pi))[0] for s in (0, 1)]).astype(float)


def _rows(r, idx, n):
    """Per-ray outputs of rays idx (numpy SoA layout [component][ray]) as one dict."""
    out = {}
    for k in KEYS:
        a = np.asarray(r[k])
        m = a.size // n
        out[k] = a.reshape(m, n)[:, idx]
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["flat", "gr"])
def test_ray_result_independent_of_batch(cfg, oracle_lib, monkeypatch):
    """(The reference batch runs on the persistent integrator, ART_SMALL_TAIL=0; the small
    batches take the default small-batch path, one wave per ray on tail_kernel.)"""
    import adiabatic_raytracer_amd as A
    p = A.Params(**CONFIGS[cfg])
    n = 1000
    s = A.sample_conversion_points(p, n, seed=1769)
    x, k, e = s["x"].reshape(3, n), s["k_init"].reshape(3, n), s["erg"]

    def run(idx):
        m = len(idx)
        r = A.propagate_batch(p, x[:, idx].ravel(), k[:, idx].ravel(), e[idx], -np.ones(m), np.full(m, -30.0),
                              np.ones(m, np.int8), max_crossings=-1, capacity=1)
        return r, m

    monkeypatch.setenv("ART_SMALL_TAIL", "0")
    full, _ = run(np.arange(n))
    monkeypatch.delenv("ART_SMALL_TAIL")
    ref = _rows(full, np.arange(n), n)
    perm = np.random.default_rng(7).permutation(n)
    batches = [np.arange(1), np.arange(63), np.arange(100, 165), np.arange(500, 757), perm]
    # slots without a crossing come back as NaN from the host entry point (include/art.h)
    empty = ref["n_cross"][0] == 0
    assert empty.any() and np.all(np.isnan(ref["xc_pos"][:, empty])) and np.all(np.isnan(ref["xc_p"][:, empty]))
    for idx in batches:
        r, m = run(idx)
        got = _rows(r, np.arange(m), m)
        for key in KEYS:
            want = ref[key][:, idx]
            assert np.array_equal(got[key], want, equal_nan=True), (cfg, len(idx), key)


@pytest.mark.gpu
def test_crossing_buffer_overflow_reports_count(oracle_lib):
    import adiabatic_raytracer_amd as A
    p = A.Params(**CONFIGS["gr"])
    n = 256
    s = A.sample_conversion_points(p, n, seed=1769)
    # the backtrace segment: axion, -k, every crossing recorded (MainRunner.jl:581-588)
    args = (s["x"], -s["k_init"], s["erg"], -np.ones(n), np.full(n, -30.0), np.zeros(n, np.int8))
    r1 = A.propagate_batch(p, *args, max_crossings=100000, capacity=1)
    r8 = A.propagate_batch(p, *args, max_crossings=100000, capacity=8)
    assert np.array_equal(r1["n_cross"], r8["n_cross"])
    assert (r1["n_cross"] > 1).any(), "no ray overflowed capacity 1"
    for key in ("xc_pos", "xc_k"):
        assert np.array_equal(r1[key].reshape(3, n), r8[key].reshape(3, 8, n)[:, 0, :], equal_nan=True)
    for key in ("xc_t", "xc_dw", "xc_p"):
        assert np.array_equal(r1[key], r8[key].reshape(8, n)[0], equal_nan=True)
    for key in ("x_end", "k_end", "status", "n_accept"):
        assert np.array_equal(r1[key], r8[key], equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["flat", "gr"])
def test_small_batch_build_matches_large_batch_build(cfg):
    """Rays of a 70000-ray batch against the same rays as a batch of 2000: bit-identical per ray
    (the second runs the 1-wave/SIMD build)."""
    import adiabatic_raytracer_amd as A
    p = A.Params(**CONFIGS[cfg])
    n, m = 70000, 2000
    s = A.sample_conversion_points(p, n, seed=1769)
    x, k, e = s["x"].reshape(3, n), s["k_init"].reshape(3, n), s["erg"]

    def run(idx):
        c = len(idx)
        return A.propagate_batch(p, x[:, idx].ravel(), k[:, idx].ravel(), e[idx], -np.ones(c), np.full(c, -30.0),
                                 np.ones(c, np.int8), max_crossings=-1, capacity=1)
    big = _rows(run(np.arange(n)), np.arange(m), n)
    small = _rows(run(np.arange(m)), np.arange(m), m)
    for key in KEYS:
        assert np.array_equal(small[key], big[key], equal_nan=True), (cfg, key)


@pytest.mark.gpu
@pytest.mark.parametrize("species", [1, 0])
def test_flat_capacity_8(species):
    """Flat batches of 2000 photons (first crossing) or backtrace axions (every crossing) with
    crossing capacity 8: the first crossing slot and the end states equal capacity 1's."""
    import adiabatic_raytracer_amd as A
    from dataclasses import replace
    p = A.Params(**CONFIGS["flat"])
    n = 2000
    s = A.sample_conversion_points(p, n, seed=1769)
    q, k, mc = (p, s["k_init"], -1) if species == 1 else (replace(p, B0=-p.B0), -s["k_init"], 100000)
    args = (s["x"], k, s["erg"], -np.ones(n), np.full(n, -30.0), np.full(n, species, np.int8))
    r1 = A.propagate_batch(q, *args, max_crossings=mc, capacity=1)
    r8 = A.propagate_batch(q, *args, max_crossings=mc, capacity=8)
    for key in ("x_end", "k_end", "status", "n_accept", "n_cross"):
        assert np.array_equal(r1[key], r8[key], equal_nan=True), key
    assert np.array_equal(r1["xc_pos"].reshape(3, n), r8["xc_pos"].reshape(3, 8, n)[:, 0, :], equal_nan=True)
    assert np.array_equal(r1["xc_p"], r8["xc_p"].reshape(8, n)[0], equal_nan=True)


_FRESH = r"""
import json, sys
import numpy as np
from dataclasses import replace
sys.path.insert(0, sys.argv[1])
import adiabatic_raytracer_amd as A
p = A.Params(theta_m=0.2, mass_a=1e-5, flat=True)
n = 2000
s = A.sample_conversion_points(p, n, seed=1769)
out = {}
for species in (1, 0):
    q, k, mc = (p, s["k_init"], -1) if species == 1 else (replace(p, B0=-p.B0), -s["k_init"], 100000)
    r = A.propagate_batch(q, s["x"], k, s["erg"], -np.ones(n), np.full(n, -30.0), np.full(n, species, np.int8),
                          max_crossings=mc, capacity=8)
    out[species] = [int(r["n_accept"].sum()), int(r["n_cross"].sum()), r["stats"]["grid"]]
print(json.dumps(out))
"""


@pytest.mark.gpu
def test_small_batch_w1_first_launch_in_fresh_process():
    """Round 2's reproducer (tools/exp_axn_case.py flat 1 2000 8, in the git history): a fresh process samples 2000
    flat roots and runs them, first as photons then as backtrace axions, with crossing capacity
    8 on the 1-wave/SIMD build. Both launches succeed, on the 1-wave grid (one block per CU)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _FRESH, root], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    for species, (acc, ncross, grid) in out.items():
        assert acc > 0 and grid == 8, (species, acc, ncross, grid)  # 2000 rays: 8 blocks of 256


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,species,cap,chunks,slots", [("flat", 1, 1, 5, 3), ("flat", 0, 3, 7, 2), ("gr", 1, 2, 4, 3)])
def test_chunked_host_pipeline_is_bit_exact(cfg, species, cap, chunks, slots, monkeypatch):
    """art_propagate_host above ART_HOST_CHUNK_MIN rays runs as a pipeline of chunks (pinned
    staging, copies overlapping the kernels, several chunks in flight with tail donation).
    An odd batch size split into uneven chunks returns exactly the single launch's outputs,
    every crossing slot included (NaN where a ray has no crossing), and the call's statistics
    are the sums over its chunks."""
    from dataclasses import replace
    import adiabatic_raytracer_amd as A
    p = A.Params(**CONFIGS[cfg])
    n = 20011
    s = A.sample_conversion_points(p, n, seed=1769)
    q, k, mc = (p, s["k_init"], -1) if species == 1 else (replace(p, B0=-p.B0), -s["k_init"], 100000)
    args = (s["x"], k, s["erg"], -np.ones(n), np.full(n, -30.0), np.full(n, species, np.int8))
    monkeypatch.setenv("ART_HOST_MODE", "single")
    ref = A.propagate_batch(q, *args, max_crossings=mc, capacity=cap, flux_nbins=50)
    monkeypatch.setenv("ART_HOST_MODE", "chunked")
    monkeypatch.setenv("ART_HOST_CHUNKS", str(chunks))
    monkeypatch.setenv("ART_HOST_SLOTS", str(slots))
    monkeypatch.setenv("ART_HOST_CHUNK_MIN", "1000")
    got = A.propagate_batch(q, *args, max_crossings=mc, capacity=cap, flux_nbins=50)
    assert np.array_equal(got["flux"], host_flux(q, got, np.full(n, species, np.int8), 50))
    for key, v in ref.items():
        if isinstance(v, np.ndarray):
            assert np.array_equal(v, got[key], equal_nan=True), (cfg, key)
    assert np.isnan(got["xc_t"].reshape(cap, n)[:, got["n_cross"] == 0]).all()
    for key in ("attempts", "accepted", "root_steps", "scan_evals", "rays", "cert_steps"):
        assert ref["stats"][key] == got["stats"][key], key


@pytest.mark.gpu
@pytest.mark.parametrize("slots", [1, 2])
def test_chunked_host_pipeline_small_chunks(slots, monkeypatch):
    """Chunks small enough for the tail kernel (<= ART_SMALL_TAIL rays, one record per ray in
    the chunk's scratch) next to larger ones, with and without tail donation (ART_HOST_SLOTS 1:
    donate = 0): the chunk's scratch slice is laid out with the launch's own small-batch
    decision, so the results are the single launch's (slot 1 overran the slice)."""
    import adiabatic_raytracer_amd as A
    p = A.Params(**CONFIGS["flat"])
    n = 3001  # chunks of ~300 (tail kernel) and ~1200 rays (persistent integrator)
    s = A.sample_conversion_points(p, n, seed=1769)
    args = (s["x"], s["k_init"], s["erg"], -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8))
    monkeypatch.setenv("ART_HOST_MODE", "single")
    ref = A.propagate_batch(p, *args, capacity=2)
    monkeypatch.setenv("ART_HOST_MODE", "chunked")
    monkeypatch.setenv("ART_HOST_CHUNKS", "4")
    monkeypatch.setenv("ART_HOST_SLOTS", str(slots))
    monkeypatch.setenv("ART_HOST_CHUNK_MIN", "1000")
    got = A.propagate_batch(p, *args, capacity=2)
    for key, v in ref.items():
        if isinstance(v, np.ndarray):
            assert np.array_equal(v, got[key], equal_nan=True), key


# the general-geometry instantiation (GEOM_ANY): boundary layer, isotropic plasma
EXTRA = {"layer": dict(theta_m=0.2, mass_a=1e-5, flat=True, bndry_lyr=1.0),
         "isotropic": dict(theta_m=0.2, mass_a=1e-5, flat=True, isotropic=True)}


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,species,cap,shift,direct", [("flat", 1, 1, 11, 0), ("flat", 0, 3, 12, 0), ("gr", 1, 2, 11, 0),
                                                           ("layer", 1, 1, 11, 0), ("isotropic", 1, 1, 12, 0),
                                                           ("flat", 0, 3, 12, 1), ("gr", 1, 2, 11, 1)])
def test_streamed_host_pipeline_is_bit_exact(cfg, species, cap, shift, direct, monkeypatch):
    """art_propagate_host's default for large batches is the streamed pipeline: one integrator
    launch over the whole batch while pieces of its inputs are still being uploaded and
    initialised (a wave waits for its rays' fresh state), each piece finalized and downloaded
    once its last ray is done (a signal the download stream waits on). With pieces of 2^11 or
    2^12 rays (10 or 5 of them) it returns exactly the single launch's outputs, every crossing
    slot included, and the same statistics. `direct`: the pieces' output blobs in pinned host
    memory, written by the helpers over PCIe (ART_HOST_DIRECT=1, no download copies)."""
    from dataclasses import replace
    import adiabatic_raytracer_amd as A
    p = A.Params(**(CONFIGS[cfg] if cfg in CONFIGS else EXTRA[cfg]))
    n = 20011
    s = A.sample_conversion_points(p, n, seed=1769)
    q, k, mc = (p, s["k_init"], -1) if species == 1 else (replace(p, B0=-p.B0), -s["k_init"], 100000)
    args = (s["x"], k, s["erg"], -np.ones(n), np.full(n, -30.0), np.full(n, species, np.int8))
    monkeypatch.setenv("ART_HOST_MODE", "single")
    ref = A.propagate_batch(q, *args, max_crossings=mc, capacity=cap, flux_nbins=50)
    monkeypatch.setenv("ART_HOST_MODE", "stream")
    monkeypatch.setenv("ART_HOST_PIECE_SHIFT", str(shift))
    monkeypatch.setenv("ART_HOST_CHUNK_MIN", "1000")
    monkeypatch.setenv("ART_HOST_DIRECT", str(direct))
    A.raytracer.host_path_counters(reset=True)
    for _ in range(2):  # the second call reuses the streams, signals and staging
        got = A.propagate_batch(q, *args, max_crossings=mc, capacity=cap, flux_nbins=50)
        for key, v in ref.items():
            if isinstance(v, np.ndarray):
                assert np.array_equal(v, got[key], equal_nan=True), (cfg, key)
        for key in ("attempts", "accepted", "root_steps", "scan_evals", "rays", "init_rhs", "cert_steps"):
            assert ref["stats"][key] == got["stats"][key], key
    # both calls streamed (no give-up: a give-up would rerun as one launch with the same outputs)
    assert A.raytracer.host_path_counters() == {"calls": 2, "streamed": 2, "stream_giveups": 0, "chunked": 0,
                                                "single": 0}
    # the device-binned flux (per piece in the streamed pipeline) is np.histogram of the outputs
    assert np.array_equal(got["flux"], host_flux(q, got, np.full(n, species, np.int8), 50))


@pytest.mark.gpu
def test_streamed_host_pipeline_gives_up_cleanly(monkeypatch):
    """A streamed call whose piece waits outlast their bound (here 0 ms) releases every wait it
    queued, lets its streams run out and runs the batch again as one launch: the results are
    the single launch's, and the next streamed call works normally."""
    import adiabatic_raytracer_amd as A
    p = A.Params(**CONFIGS["flat"])
    n = 20011
    s = A.sample_conversion_points(p, n, seed=1769)
    args = (s["x"], s["k_init"], s["erg"], -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8))
    monkeypatch.setenv("ART_HOST_MODE", "single")
    ref = A.propagate_batch(p, *args)
    monkeypatch.setenv("ART_HOST_MODE", "stream")
    monkeypatch.setenv("ART_HOST_PIECE_SHIFT", "11")
    monkeypatch.setenv("ART_HOST_CHUNK_MIN", "1000")
    A.raytracer.host_path_counters(reset=True)
    for limit, want in (("0", {"streamed": 0, "stream_giveups": 1, "single": 1}),
                        ("30000", {"streamed": 1, "stream_giveups": 1, "single": 1})):
        monkeypatch.setenv("ART_HOST_STREAM_TIMEOUT_MS", limit)
        got = A.propagate_batch(p, *args)
        for key, v in ref.items():
            if isinstance(v, np.ndarray):
                assert np.array_equal(v, got[key], equal_nan=True), (limit, key)
        # the give-up is visible to the caller (art_host_path_counters), not only on stderr
        cnt = A.raytracer.host_path_counters()
        assert {k: cnt[k] for k in want} == want, (limit, cnt)


@pytest.mark.gpu
def test_streamed_host_pipeline_device_give_up(monkeypatch):
    """The device side's bound: with the second upload unit held back 1.5 s and the waves' bound
    on a chunk flag at 0.2 s, the integrator's waves outwait it, raise the abort word and stop;
    the host sees it,
    lets the launch run out and runs the batch again as one launch. The results are the single
    launch's, the give-up is counted, and the next streamed call works normally."""
    import adiabatic_raytracer_amd as A
    p = A.Params(**CONFIGS["flat"])
    n = 20011
    s = A.sample_conversion_points(p, n, seed=1769)
    args = (s["x"], s["k_init"], s["erg"], -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8))
    monkeypatch.setenv("ART_HOST_MODE", "single")
    ref = A.propagate_batch(p, *args)
    monkeypatch.setenv("ART_HOST_MODE", "stream")
    monkeypatch.setenv("ART_HOST_PIECE_SHIFT", "11")
    monkeypatch.setenv("ART_HOST_CHUNK_MIN", "1000")
    A.raytracer.host_path_counters(reset=True)
    monkeypatch.setenv("ART_HOST_WAVE_WAIT_MS", "200")
    monkeypatch.setenv("ART_HOST_INIT_RAYS", "512")  # (the integrator starts before the held-back unit)
    monkeypatch.setenv("ART_HOST_FIRST_UNIT", "1024")
    monkeypatch.setenv("ART_HOST_UNIT", "4096")
    import time
    for delay, want in (("1500", {"streamed": 0, "stream_giveups": 1, "single": 1}),
                        ("0", {"streamed": 1, "stream_giveups": 1, "single": 1})):
        monkeypatch.setenv("ART_HOST_UPLOAD_DELAY_MS", delay)
        t0 = time.perf_counter()
        got = A.propagate_batch(p, *args)
        wall = time.perf_counter() - t0
        # the abandoned launch stops at once (the helpers drain its queue on the abort word, and
        # the ready counter is not raised past the landed inputs): the call costs the held-back
        # upload plus the rerun, not a second pass over the batch
        assert wall < float(delay) / 1e3 + 1.0, (delay, wall)
        for key, v in ref.items():
            if isinstance(v, np.ndarray):
                assert np.array_equal(v, got[key], equal_nan=True), (delay, key)
        cnt = A.raytracer.host_path_counters()
        assert {k: cnt[k] for k in want} == want, (delay, cnt)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,species,cap", [("flat", 1, 1), ("gr", 1, 1), ("gr_oblique", 1, 2), ("flat", 0, 3)])
def test_small_batch_tail_mode_is_bit_exact(cfg, species, cap, monkeypatch):
    """Batches of at most one ray per SIMD (ART_SMALL_TAIL, default 1024 on the MI355X) run every
    ray on a wave of its own (tail_kernel, fed by pack_fresh_kernel) instead of a lane of the
    persistent integrator: every output, crossing slot and launch counter is the same bit for
    bit, forward photons and all-crossings axion backtraces (MainRunner.jl:581-591) alike."""
    from dataclasses import replace
    import adiabatic_raytracer_amd as A
    p = A.Params(**CONFIGS[cfg])
    n = 777
    s = A.sample_conversion_points(p, n, seed=1769)
    q, k, mc = (p, s["k_init"], -1) if species == 1 else (replace(p, B0=-p.B0), -s["k_init"], 100000)
    args = (s["x"], k, s["erg"], -np.ones(n), np.full(n, -30.0), np.full(n, species, np.int8))
    monkeypatch.setenv("ART_SMALL_TAIL", "0")
    ref = A.propagate_batch(q, *args, max_crossings=mc, capacity=cap)
    monkeypatch.setenv("ART_SMALL_TAIL", "1024")
    got = A.propagate_batch(q, *args, max_crossings=mc, capacity=cap)
    for key, v in ref.items():
        if isinstance(v, np.ndarray):
            assert np.array_equal(v, got[key], equal_nan=True), (cfg, key)
    # (interp_evals counts the interpolant evaluations a kernel actually performs: the tail
    # kernel keeps all 49 grid values of a step in its lanes and re-evaluates fewer)
    for key in ("attempts", "accepted", "root_steps", "scan_evals", "rays", "init_rhs", "cert_steps"):
        assert ref["stats"][key] == got["stats"][key], key
    assert got["stats"]["interp_evals"] <= ref["stats"]["interp_evals"]
