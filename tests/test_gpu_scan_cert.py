"""The certified-negative resonance scan (art_core.h scan_certified_negative)
skips the grid evaluations of steps whose 49 sign codes are provably "negative". It must
change nothing: the kernel with the certificate (default) and without it (ART_SCAN_CERT=0)
produce bit-identical segments -- end states, statuses, step counts, crossings and P --
while evaluating fewer grid points."""
import numpy as np
import pytest

from conftest import CONFIGS

pytestmark = pytest.mark.gpu

KEYS = ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept", "n_reject", "n_cross", "xc_pos", "xc_k",
        "xc_t", "xc_dw", "xc_p")


def _run(p, s, n, species, max_crossings, cap):
    import adiabatic_raytracer_amd as A
    k0 = s["k_init"] if species == 1 else -s["k_init"]
    return A.propagate_batch(p, s["x"], k0, s["erg"], -np.ones(n), np.full(n, -30.0), np.full(n, species, np.int8),
                             max_crossings=max_crossings, capacity=cap)


@pytest.mark.parametrize("cfg,species", [("flat", 1), ("gr", 1), ("gr_oblique", 1), ("gr", 0)])
def test_certificate_is_bit_exact(cfg, species, monkeypatch):
    import adiabatic_raytracer_amd as A
    from dataclasses import replace
    p = A.Params(**CONFIGS[cfg])
    if species == 0:  # backtrace: axion, -k, -B0, every crossing (MainRunner.jl:578-590)
        p = replace(p, B0=-p.B0)
    n = 20000 if species == 1 else 4000
    s = A.sample_conversion_points(A.Params(**CONFIGS[cfg]), n, seed=1769)
    mc, cap = (-1, 1) if species == 1 else (100000, 8)
    a = _run(p, s, n, species, mc, cap)
    monkeypatch.setenv("ART_SCAN_CERT", "0")
    b = _run(p, s, n, species, mc, cap)
    for k in KEYS:
        assert np.array_equal(a[k], b[k], equal_nan=True), (cfg, k)
    sa, sb = a["stats"], b["stats"]
    assert sb["cert_steps"] == 0 and sa["cert_steps"] > 0, (sa, sb)
    assert sa["accepted"] == sb["accepted"] and sa["scan_evals"] < sb["scan_evals"], (sa, sb)
    print(cfg, species, "certified", sa["cert_steps"] / sa["accepted"], "scan evals", sa["scan_evals"] / sb["scan_evals"])


@pytest.mark.parametrize("cfg", ["flat", "gr", "scan7"])
def test_sampler_certificate_is_bit_exact(cfg, monkeypatch):
    """The sampler's certified-negative steps (sample_kernel; a step whose every point is
    provably below the resonance evaluates only its last point) change no sample: positions,
    momenta, energies, weights and attempt counts with and without them (ART_SCAN_CERT=0)
    are bit-identical, for the flat and GR geometries and the heaviest scan point."""
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd.scan import scan_grid
    kw = scan_grid()[7] if cfg == "scan7" else CONFIGS[cfg]
    p = A.Params(**kw)
    n = 20000 if cfg != "scan7" else 4000
    a = A.sample_conversion_points(p, n, seed=1769)
    monkeypatch.setenv("ART_SCAN_CERT", "0")
    b = A.sample_conversion_points(p, n, seed=1769)
    for k in ("x", "k_init", "erg", "vifty", "weights", "attempts"):
        assert np.array_equal(a[k], b[k], equal_nan=True), (cfg, k)


@pytest.mark.parametrize("cfg", ["flat", "scan_longest"])
def test_sampler_waves_are_bit_exact(cfg):
    """art_set_sampler_waves (include/art.h) only picks the sampler's build: the 3-wave build for
    every line (what the scan takes with samplers in flight), the 2-wave one and the default choice
    by line length give bit-identical samples, for short lines (step by step) and the scan's long
    ones (blocks of steps at 2 waves by default)."""
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    from adiabatic_raytracer_amd.scan import scan_grid
    kw = max(scan_grid(), key=lambda g: A.Params(**g).max_r()) if cfg == "scan_longest" else CONFIGS[cfg]
    eng = Engine(A.Params(**kw))
    n = 20000 if cfg == "flat" else 4000
    out = {}
    try:
        for w in (0, 3, 2):
            eng.set_sampler_waves(w)
            s = eng.sample(n, seed=1769)
            out[w] = {k: v.cpu().numpy() for k, v in s.items()}
    finally:
        eng.set_sampler_waves(0)
    for w in (3, 2):
        for k in ("x", "k_init", "erg", "vifty", "weights", "attempts"):
            assert np.array_equal(out[0][k], out[w][k], equal_nan=True), (cfg, w, k)
