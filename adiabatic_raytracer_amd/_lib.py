"""ctypes binding of libart.so (include/art.h). Fails loudly when the library is missing:
there is no CPU fallback anywhere in the product path."""
import ctypes as C
import os

from .build import LIB

ART_VERN6, ART_RK4 = 0, 1
ART_AXION, ART_PHOTON = 0, 1
STATUS_NAMES = {0: "Success", 1: "Terminated(crossing)", 2: "Terminated(hit NS)", 3: "MaxIters", 4: "NonFinite"}


class ArtParams(C.Structure):
    _fields_ = [
        ("theta_m", C.c_double), ("omega_pul", C.c_double), ("B0", C.c_double), ("rNS", C.c_double),
        ("mass_ns", C.c_double), ("mass_a", C.c_double), ("g_agg", C.c_double), ("bndry_lyr", C.c_double),
        ("ln_t_end", C.c_double), ("abstol", C.c_double), ("reltol", C.c_double), ("dtmin", C.c_double),
        ("maxiters", C.c_int64), ("flat", C.c_int32), ("isotropic", C.c_int32), ("melrose", C.c_int32),
        ("integrator", C.c_int32), ("n_fixed", C.c_int32), ("interp_points", C.c_int32),
    ]


class SegmentOut(C.Structure):
    _fields_ = [("x_end", C.c_void_p), ("k_end", C.c_void_p), ("u7_end", C.c_void_p), ("tau_end", C.c_void_p),
                ("status", C.c_void_p), ("n_accept", C.c_void_p), ("n_reject", C.c_void_p)]


class CrossingBuf(C.Structure):
    _fields_ = [("capacity", C.c_int32), ("count", C.c_void_p), ("pos", C.c_void_p), ("k", C.c_void_p),
                ("t", C.c_void_p), ("dw", C.c_void_p), ("p_nonad", C.c_void_p)]


# name -> (restype, argtypes); the test suite checks this table against include/art.h
class TreeOpts(C.Structure):  # include/art.h art_tree_opts
    _fields_ = [("num_cutoff", C.c_int32), ("mc_nodes", C.c_int32), ("max_nodes", C.c_int32),
                ("splittings_cutoff", C.c_int32), ("crossing_cap", C.c_int32), ("tree_offset", C.c_int32),
                ("prob_cutoff", C.c_double), ("seed", C.c_uint64)]


class TreeTraj(C.Structure):  # include/art.h art_tree_traj
    _fields_ = [("ntimes", C.c_int32), ("crossing_cap", C.c_int32), ("traj", C.c_void_p), ("times", C.c_void_p),
                ("count", C.c_void_p), ("xc", C.c_void_p)]


_P = C.POINTER(ArtParams)
_v = C.c_void_p
_i64, _i32, _d, _u64 = C.c_int64, C.c_int32, C.c_double, C.c_uint64
SIGNATURES = {
    "art_abi_version": (C.c_int, []),
    "art_last_error": (C.c_char_p, []),
    "art_device_count": (C.c_int, [C.POINTER(C.c_int32)]),
    "art_set_device": (C.c_int, [_i32]),
    "art_synchronize": (C.c_int, []),
    "art_shutdown": (C.c_int, []),
    "art_last_kernel_ms": (C.c_double, []),
    "art_last_stats": (C.c_int, [C.POINTER(C.c_uint64), C.POINTER(C.c_int32)]),
    "art_vern6_tableau": (C.c_int, [_v, _v, _v, _v]),
    "art_find_conversion_surface": (C.c_double, [_P]),
    "art_propagate_host": (C.c_int, [_P, _i64, _v, _v, _v, _v, _v, _v, _i32, C.POINTER(SegmentOut),
                                     C.POINTER(CrossingBuf)]),
    "art_propagate_device": (C.c_int, [_P, _i64, _v, _v, _v, _v, _v, _v, _i32, C.POINTER(SegmentOut),
                                       C.POINTER(CrossingBuf), _v]),
    "art_propagate_host_flux": (C.c_int, [_P, _i64, _v, _v, _v, _v, _v, _v, _i32, C.POINTER(SegmentOut),
                                          C.POINTER(CrossingBuf), _i32, _v]),
    "art_propagate_host_flux_async": (C.c_int, [_P, _i64, _v, _v, _v, _v, _v, _v, _i32, C.POINTER(SegmentOut),
                                                C.POINTER(CrossingBuf), _i32, _v, C.POINTER(C.c_int64)]),
    "art_host_wait": (C.c_int, [C.c_int64]),
    "art_host_path_counters": (C.c_int, [_v, _i32, _i32]),
    "art_propagate_traj_host": (C.c_int, [_P, _i64, _v, _v, _v, _v, _v, _v, _i32, C.POINTER(SegmentOut),
                                          C.POINTER(CrossingBuf), _i32, _v, _v, _v]),
    "art_propagate_traj_device": (C.c_int, [_P, _i64, _v, _v, _v, _v, _v, _v, _i32, C.POINTER(SegmentOut),
                                            C.POINTER(CrossingBuf), _i32, _v, _v, _v, _v]),
    "art_get_prob_nonad_host": (C.c_int, [_P, _i64, _v, _v, _v, _i64, _v, _v]),
    "art_get_prob_nonad_device": (C.c_int, [_P, _i64, _v, _v, _v, _i64, _v, _v, _v]),
    "art_sample_conversion_points_host": (C.c_int, [_P, _d, _u64, _i64, _i64, _v, _v, _v, _v, _v, _v]),
    "art_sample_conversion_points_device": (C.c_int, [_P, _d, _u64, _i64, _i64, _v, _v, _v, _v, _v, _v, _v]),
    "art_flux_histogram_device": (C.c_int, [_P, _i64, _v, _v, _v, _v, _v, _i32, _v, _v]),
    "art_grow_trees": (C.c_int, [_P, _i64, _v, _v, _v, _v, C.POINTER(TreeOpts), _i64, _v, C.POINTER(_i64), _v, _v]),
    "art_grow_trees_traj": (C.c_int, [_P, _i64, _v, _v, _v, _v, C.POINTER(TreeOpts), _i64, _v, C.POINTER(_i64), _v,
                                      _v, C.POINTER(TreeTraj)]),
    "art_event_weight_host": (C.c_int, [_P, _d, _d, _d, _i64, _v, _v, _v, _v]),
    "art_event_weight_device": (C.c_int, [_P, _d, _d, _d, _i64, _v, _v, _v, _v, _v]),
    "art_recent_kernel_ms": (C.c_int, [_i32, _v]),
    "art_recent_kernel_span_ms": (C.c_int, [_i32, _v]),
    "art_set_tail_donation": (C.c_int, [_i32]),
    "art_set_graduation": (C.c_int, [_i32]),
    "art_set_sampler_waves": (C.c_int, [_i32]),
    "art_flux_histogram_phi_device": (C.c_int, [_i64, _v, _v, _v, _i32, _v, _v]),
    "art_flux_histogram_phi_range_device": (C.c_int, [_i64, _v, _v, _v, _i32, _d, _d, _v, _v]),
    "art_comm_unique_id": (C.c_int, [_v]),
    "art_comm_init": (C.c_int, [_i32, _i32, _v]),
    "art_flux_allreduce": (C.c_int, [_v, _i64, _v]),
    "art_flux_allreduce_host": (C.c_int, [_v, _i64]),
    "art_comm_destroy": (C.c_int, []),
    "art_eval_rhs_device": (C.c_int, [_P, _i64, _v, _v, _v, _v, _v, _v]),
    "art_eval_hamiltonian_device": (C.c_int, [_P, _i64, _v, _v, _v, _v, _v, _v, _v, _v, _v]),
    "art_eval_condition_device": (C.c_int, [_P, _i64, _v, _v, _v, _v]),
}

_lib = None


class ArtError(RuntimeError):
    pass


def load(path=None):
    """Load libart.so; raise if it is absent (build it with `python -m adiabatic_raytracer_amd.build`)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("ART_LIB", LIB)
    if not os.path.exists(path):
        raise ArtError(f"libart.so not found at {path}: the HIP engine must be built "
                       f"(python -m adiabatic_raytracer_amd.build); there is no CPU fallback")
    # PyTorch ships its own HIP runtime under the same soname (libamdhip64.so.7). Whichever is
    # loaded first serves the whole process; torch refuses a foreign one ("No HIP GPUs are
    # available"), so when torch is present it is imported first and libart binds to torch's.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc):
    if rc != 0:
        raise ArtError(f"libart error {rc}: {load().art_last_error().decode()}")
    return rc
