"""The build's npy rows against the reference's own post-processing, run on them.

tests/golden/combine_py/ holds (tests/golden/make_combine_fixture.py):
  * input_mode{0,1}_{0,1}.npy: npy row files the GPU build wrote (trees.main_runner_tree,
    two independent runs as two --ftag processes would, saveMode 0 and 1);
  * expected_mode{0,1}.npy: what the reference's Combine_Files.py, run unchanged on those
    files in this container, wrote.
This pins the 13- and 29-column layout (MainRunner.jl:715,720), the event-number offset
(Combine_Files.py:22) and the division of column 10 by the number of files (:28), and checks
that the build's restatement trees.combine_files_py reproduces the reference bit for bit."""
import os

import numpy as np
import pytest

G = os.path.join(os.path.dirname(__file__), "golden", "combine_py")
pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(G, "expected_mode0.npy")),
                                reason="fixtures not generated")


@pytest.mark.parametrize("mode,ncol", [(0, 13), (1, 29)])
def test_layout_and_reference_combine(mode, ncol, tmp_path):
    from adiabatic_raytracer_amd.trees import combine_files_py
    ins = [np.load(os.path.join(G, f"input_mode{mode}_{k}.npy")) for k in (0, 1)]
    exp = np.load(os.path.join(G, f"expected_mode{mode}.npy"))
    for a in ins:
        assert a.ndim == 2 and a.shape[1] == ncol and a.dtype == np.float64
        ev = a[:, 0]
        assert np.all(ev == np.round(ev)) and np.all(ev >= 1) and np.all(np.diff(ev) >= 0)  # event numbers
        assert set(np.unique(a[:, 1])) <= {0.0, 1.0}  # particle id: axion 0, photon 1
        assert np.all(a[:, 7] > 0) and np.all(a[:, 8] > 0)  # sln_prob / f_inx, weight
    # what Combine_Files.py did to them
    assert exp.shape == (ins[0].shape[0] + ins[1].shape[0], ncol)
    assert np.array_equal(exp[:len(ins[0]), 0], ins[0][:, 0])
    assert np.array_equal(exp[len(ins[0]):, 0], ins[1][:, 0] + ins[0][-1, 0])  # :22 offset
    assert np.array_equal(exp[:, 9], np.concatenate([ins[0][:, 9], ins[1][:, 9]]) / 2)  # :28 quirk
    other = [c for c in range(ncol) if c not in (0, 9)]
    assert np.array_equal(exp[:, other], np.concatenate(ins)[:, other])
    # the build's restatement reproduces the reference's output bit for bit
    files = []
    names = open(os.path.join(G, f"names_mode{mode}.txt")).read().split()
    for k, a in enumerate(ins):
        f = tmp_path / names[k]
        np.save(f, a)
        files.append(str(f))
    got = combine_files_py(str(tmp_path / "combined.npy"), files)
    assert np.array_equal(got, exp, equal_nan=True)
    assert np.array_equal(np.load(tmp_path / "combined.npy"), exp, equal_nan=True)
