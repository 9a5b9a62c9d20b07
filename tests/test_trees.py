"""Host side of the tree driver and event loop (MainRunner.jl:126-761) on CPU: the node
record layout of the C ABI, the reference's npy file name, and the oracle's sequential
get_tree / main_runner_tree restatement (oracle/tree.py) that the GPU tests check against."""
import ctypes as C

import numpy as np

from adiabatic_raytracer_amd.trees import NODE_DTYPE, TreeOpts, tree_file_name


class _CNode(C.Structure):  # include/art.h art_tree_node, field by field
    _fields_ = [("tree", C.c_int32), ("species", C.c_int32), ("is_final", C.c_int32), ("n_cross", C.c_int32),
                ("status", C.c_int32), ("pad", C.c_int32)] + [
        (n, C.c_double) for n in ("weight", "prob", "parent_weight", "prob_conv", "prob_conv0")] + [
        ("x0", C.c_double * 3), ("k0", C.c_double * 3), ("t0", C.c_double), ("dw0", C.c_double),
        ("x_end", C.c_double * 3), ("k_end", C.c_double * 3), ("u7_end", C.c_double), ("tau_end", C.c_double),
        ("xc", C.c_double * 3), ("kc", C.c_double * 3), ("tc", C.c_double), ("dwc", C.c_double), ("pc", C.c_double)]


def test_node_record_matches_c_layout():
    assert NODE_DTYPE.itemsize == C.sizeof(_CNode)
    for name, _ in _CNode._fields_:
        assert NODE_DTYPE.fields[name][1] == getattr(_CNode, name).offset, name
    assert C.sizeof(TreeOpts) == 40


def test_tree_file_name_matches_reference_format():
    # the reference's own analysis scripts load names like this (jonas_test_analyses/npz_example.py)
    f = tree_file_name("results", 2e-5, 1e-18, 0.2, 1.0, 1e14, 10, 1000, 5, 5, 5, "test0")
    assert f == ("results/npy/tree_MassAx_2.0e-5_AxionG_1.0e-18_ThetaM_0.2_rotPulsar_1.0_B0_1.0e14_Ax_trajs_10"
                 "_N_Times_1000_num_cutoff_5_MC_nodes_5_max_nodes_5_test0.npy")
    assert "_B0_2.5e13_" in tree_file_name("r", 1e-6, 1e-12, 0.0, 6.283185307179586, 2.5e13, 3, 3, 5, 5, 50, "")
    assert "_rotPulsar_6.283185307179586_" in tree_file_name("r", 1e-6, 1e-12, 0.0, 6.283185307179586, 2.5e13, 3, 3,
                                                             5, 5, 50, "")


def test_oracle_event_loop_rows(oracle_lib):
    from oracle import tree as T
    p = oracle_lib.make_params(theta_m=0.2, mass_a=1e-5, flat=True)
    rows = T.main_runner_rows(p, 9, saveMode=1)
    assert rows.shape[1] == 29 and rows.shape[0] >= 8
    assert np.all(np.diff(rows[:, 0]) >= 0) and set(np.unique(rows[:, 1])) <= {0.0, 1.0}
    assert np.all(rows[:, 8] > 0) and np.all(rows[:, 8] <= 1.0)          # weights are probabilities
    assert np.all(np.abs(rows[:, 8] - rows[:, 13]) == 0)                 # weight_tmp == tree.weight
    assert np.all(rows[:, 14] == 0) and np.all(rows[:, 15] == 1)         # opticalDepth, weightC
    again = T.main_runner_rows(p, 9, saveMode=1)
    assert np.array_equal(rows, again)                                    # Philox: reproducible
    short = T.main_runner_rows(p, 9, saveMode=0)
    assert short.shape[1] == 13 and np.array_equal(short, rows[:, :13])


def test_oracle_full_tree_weights_conserve(oracle_lib):
    """Full-tree mode (MC never triggers): each split divides the parent weight between its
    two children, so the popped + pending weights always add up to the root's."""
    from oracle import tree as T
    p = oracle_lib.make_params(theta_m=0.2, mass_a=1e-5, flat=True)
    s = oracle_lib.sample(p, oracle_lib.find_conversion_surface(p), 1769, 0, 4, nthreads=1)
    x, k = s["x"].reshape(3, 4).T, s["k_init"].reshape(3, 4).T
    for i in range(4):
        root = T.Node(x[i].copy(), k[i].copy(), 0.0, -1.0, T.PHOTON, 1.0, 1.0, -1.0, -1.0, -1.0)
        tree, count, info = T.get_tree(p, root, s["erg"][i], i, num_cutoff=5, MC_nodes=1000, max_nodes=50)
        assert info > 0 and count == len(tree)
        leaves = sum(e.weight for e in tree if not e.xc)
        assert leaves <= 1.0 + 1e-12
