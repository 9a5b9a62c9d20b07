"""Saved trajectory points (saveat, RayTracer.jl:176, 383, 427-444; art_propagate_traj_*) and the
saveMode 3 tree dumps built on them (saveNode, MainRunner.jl:17-65, :573-612, :671).

The saved points are the start, the interior times ln t0 + k (ln t_end - ln t0)/(ntimes - 1)
the segment reached, and its end. The interior ones come from the step's cubic Hermite
interpolant (the reference interpolates with Vern6's own 6th-order dense output, which is not
available here -- a documented deviation), so they are checked against the ORACLE run
stopped exactly at that time with a tolerance for the interpolant: median relative position
error <= 1e-6 and 95th percentile <= 1e-3."""
import numpy as np
import pytest

from conftest import CONFIGS

pytestmark = pytest.mark.gpu


def _sample(A, kw, n):
    p = A.Params(**kw)
    return p, A.sample_conversion_points(p, n, seed=1769)


@pytest.mark.parametrize("cfg,ntimes", [("flat", 3), ("gr", 7)])
def test_saved_points_structure(cfg, ntimes):
    import adiabatic_raytracer_amd as A
    n = 2000
    p, s = _sample(A, CONFIGS[cfg], n)
    g = A.propagate_batch(p, s["x"], s["k_init"], s["erg"], -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8),
                          max_crossings=-1, ntimes=ntimes)
    plain = A.propagate_batch(p, s["x"], s["k_init"], s["erg"], -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8),
                              max_crossings=-1)
    for key in ("x_end", "status", "n_accept", "xc_pos"):  # saving changes nothing else
        assert np.array_equal(g[key], plain[key], equal_nan=True), key  # (xc_pos NaN: no crossing)
    cnt, tr, tt = g["traj_n"], g["traj"], g["traj_t"]
    assert np.all((cnt >= 2) & (cnt <= ntimes))
    ok = g["status"] == 0
    assert np.all(cnt[ok] == ntimes) and np.all(tt[ntimes - 1, ok] == p.to_c().ln_t_end)
    x0 = s["x"].reshape(3, n)
    assert np.allclose(tr[:, 0, :], x0, rtol=1e-12, atol=1e-9)
    idx = np.arange(n)
    assert np.array_equal(tr[:, cnt - 1, idx], g["x_end"].reshape(3, n))
    D = (p.to_c().ln_t_end + 30.0) / (ntimes - 1)
    for i in range(n):
        t = tt[:cnt[i], i]
        assert t[0] == -30.0 and np.all(np.diff(t) >= 0.0)
        assert np.allclose(t[1:-1], -30.0 + D * np.arange(1, cnt[i] - 1), rtol=0, atol=1e-12)


def test_interior_points_match_the_oracle(oracle_lib):
    import adiabatic_raytracer_amd as A
    kw, ntimes, n = CONFIGS["flat"], 5, 256
    p, s = _sample(A, kw, n)
    g = A.propagate_batch(p, s["x"], s["k_init"], s["erg"], -np.ones(n), np.full(n, -30.0), np.ones(n, np.int8),
                          max_crossings=-1, ntimes=ntimes)
    errs = []
    for k in range(1, ntimes - 1):
        sel = np.flatnonzero(g["traj_n"] > k + 1)
        tk = g["traj_t"][k, sel[0]]
        po = oracle_lib.make_params(ln_t_end=float(tk), **kw)
        xs = s["x"].reshape(3, n)[:, sel].reshape(-1)
        ks = s["k_init"].reshape(3, n)[:, sel].reshape(-1)
        o = oracle_lib.propagate(po, xs, ks, s["erg"][sel], -1.0, -30.0, 1, max_crossings=-1)
        fine = o["status"] == 0  # reached t_k without a crossing, as the GPU segment did
        xo = o["x_end"].reshape(3, -1)[:, fine]
        xg = g["traj"][:, k, sel[fine]]
        errs.extend(np.abs(xg - xo).max(0) / np.linalg.norm(xo, axis=0))
    errs = np.asarray(errs)
    assert errs.size > 50
    assert np.median(errs) <= 1e-6 and np.percentile(errs, 95) <= 1e-3, np.percentile(errs, [50, 90, 95, 100])


def test_save_mode_3_tree_files(tmp_path):
    import adiabatic_raytracer_amd as A
    p = A.Params(**CONFIGS["flat"])
    n_ev = 6
    rows = A.trees.main_runner_tree(p, n_ev + 1, saveMode=3, ntimes=3, dir_tag=str(tmp_path), file_tag="s")
    assert len(rows)
    for e in range(1, n_ev + 1):
        lines = (tmp_path / "tree" / f"tree_s{e}").read_text().split("\n")
        assert lines[-1] == ""
        lines, i, nblocks = lines[:-1], 0, 0
        while i < len(lines):  # header, 3 "-" lines or 4 crossing lines (x, y, z, tc), 4 trajectory lines
            sp, w, pr, pw = lines[i].split()
            assert sp in ("photon", "axion") and float(w) >= 0.0
            if nblocks == 0:
                assert sp == "axion"  # the backtrace node comes first (MainRunner.jl:612)
            if lines[i + 1] == "-":
                assert lines[i + 2] == "-" and lines[i + 3] == "-"
                i += 4
            else:
                assert len({len(lines[i + j].split()) for j in (1, 2, 3, 4)}) == 1
                i += 5
            cols = [np.array(lines[i + j].split(), float) for j in range(4)]
            assert len({c.size for c in cols}) == 1 and 2 <= cols[0].size <= 3
            assert np.all(np.diff(cols[3]) >= 0.0)
            i += 4
            nblocks += 1
        assert nblocks >= 2
