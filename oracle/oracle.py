"""ctypes binding of oracle/build/liboracle.so (TEST INFRASTRUCTURE ONLY).

Every function mirrors a reference function (RayTracer.jl / MainRunner.jl file:line
in art_oracle.cpp). Arrays follow the product's C ABI layout: structure-of-arrays,
identical to a Julia column-major N x 3 matrix.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

ART_VERN6, ART_RK4 = 0, 1
ART_AXION, ART_PHOTON = 0, 1


class ArtParams(C.Structure):
    """Same layout as `art_params` in include/art.h."""
    _fields_ = [
        ("theta_m", C.c_double), ("omega_pul", C.c_double), ("B0", C.c_double), ("rNS", C.c_double),
        ("mass_ns", C.c_double), ("mass_a", C.c_double), ("g_agg", C.c_double), ("bndry_lyr", C.c_double),
        ("ln_t_end", C.c_double), ("abstol", C.c_double), ("reltol", C.c_double), ("dtmin", C.c_double),
        ("maxiters", C.c_int64), ("flat", C.c_int32), ("isotropic", C.c_int32), ("melrose", C.c_int32),
        ("integrator", C.c_int32), ("n_fixed", C.c_int32), ("interp_points", C.c_int32),
    ]


def make_params(theta_m=0.0, omega_pul=1.0, B0=1e14, rNS=10.0, mass_ns=1.0, mass_a=1e-5, g_agg=1e-12,
                bndry_lyr=-1.0, ln_t_end=None, abstol=1e-6, reltol=1e-7, dtmin=1e-13, maxiters=100000,
                flat=False, isotropic=False, integrator=ART_VERN6, n_fixed=2000, interp_points=50):
    if ln_t_end is None:
        ln_t_end = float(np.log(1.0 / omega_pul))
    return ArtParams(theta_m, omega_pul, B0, rNS, mass_ns, mass_a, g_agg, bndry_lyr, ln_t_end, abstol, reltol,
                     dtmin, maxiters, int(flat), int(isotropic), 1, integrator, n_fixed, interp_points)


def build():
    src = os.path.join(_HERE, "art_oracle.cpp")
    if (not os.path.exists(_LIB_PATH)) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = C.CDLL(_LIB_PATH)
        P = C.POINTER
        d, i32, i64, u64 = C.c_double, C.c_int32, C.c_int64, C.c_uint64
        pd, pi32, pi8, pu32 = P(d), P(i32), P(C.c_int8), P(C.c_uint32)
        pp = P(ArtParams)
        sig = {
            "oracle_philox4x32_10": (None, [pu32, pu32, pu32]),
            "oracle_attempt_uniforms": (None, [u64, u64, C.c_uint32, pd]),
            "oracle_vern6_tableau": (None, [pd, pd, pd, pd]),
            "oracle_metric": (None, [d, d, d, pd]),
            "oracle_omega_p": (d, [pp, d, d, d, d, C.c_int, d]),
            "oracle_hamiltonian": (None, [pp, pd, pd, d, d, pd, pd, pd, pd]),
            "oracle_rhs": (None, [pp, C.c_int, pd, d, d, pd]),
            "oracle_condition": (d, [pp, pd, d]),
            "oracle_initial_state": (None, [pp, pd, pd, d, d, pd]),
            "oracle_back_transform": (None, [pp, pd, d, pd, pd]),
            "oracle_find_conversion_surface": (d, [pp]),
            "oracle_get_prob_nonad": (None, [pp, i64, pd, pd, pd, i64, P(i64), pd]),
            "oracle_event_weight": (None, [pp, i64, pd, pd, pd, C.c_double, C.c_double, C.c_double, pd]),
            "oracle_propagate": (None, [pp, i64, pd, pd, pd, pd, pd, pi8, i32, pd, pd, pd, pd, pi32, pi32, pi32,
                                        i32, pi32, pd, pd, pd, pd, pd, i32]),
            "oracle_sample": (None, [pp, d, u64, i64, i64, pd, pd, pd, pd, pi32, pi32, i32]),
            "oracle_sampler_condition": (d, [pp, pd, pd, d]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(_lib, name)
            fn.restype = res
            fn.argtypes = args
    return _lib


def _pd(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _arr(a, dtype=np.float64):
    return np.ascontiguousarray(a, dtype=dtype)


def philox4x32_10(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().oracle_philox4x32_10(c, k, o)
    return list(o)


def vern6_tableau():
    c, A, b, bh = (np.zeros(9), np.zeros(81), np.zeros(9), np.zeros(9))
    lib().oracle_vern6_tableau(_pd(c), _pd(A), _pd(b), _pd(bh))
    return c, A.reshape(9, 9), b, bh


def metric(r, th, mass_ns):
    g = np.zeros(4)
    lib().oracle_metric(r, th, mass_ns, _pd(g))
    return g


def omega_p(p, r, th, ph, t, zeroIn, bndry):
    return lib().oracle_omega_p(C.byref(p), r, th, ph, t, int(zeroIn), bndry)


def hamiltonian(p, x, k, T, E):
    x, k = _arr(x), _arr(k)
    H, gx, gk, gT = np.zeros(1), np.zeros(3), np.zeros(3), np.zeros(1)
    lib().oracle_hamiltonian(C.byref(p), _pd(x), _pd(k), T, E, _pd(H), _pd(gx), _pd(gk), _pd(gT))
    return H[0], gx, gk, gT[0]


def rhs(p, species, u, tau, erg):
    u = _arr(u)
    du = np.zeros(7)
    lib().oracle_rhs(C.byref(p), species, _pd(u), tau, erg, _pd(du))
    return du


def condition(p, u, tau):
    return lib().oracle_condition(C.byref(p), _pd(_arr(u)), tau)


def initial_state(p, x0, k0, erg, dw):
    u0 = np.zeros(7)
    lib().oracle_initial_state(C.byref(p), _pd(_arr(x0)), _pd(_arr(k0)), erg, dw, _pd(u0))
    return u0


def find_conversion_surface(p):
    return lib().oracle_find_conversion_surface(C.byref(p))


def get_prob_nonad(p, pos, kpos, erg_eff, group_start=None):
    pos, kpos, erg_eff = _arr(pos).reshape(-1), _arr(kpos).reshape(-1), _arr(erg_eff).reshape(-1)
    nc = erg_eff.size
    out = np.zeros(nc)
    if group_start is None:
        lib().oracle_get_prob_nonad(C.byref(p), nc, _pd(pos), _pd(kpos), _pd(erg_eff), nc, None, _pd(out))
    else:
        gs = _arr(group_start, np.int64)
        lib().oracle_get_prob_nonad(C.byref(p), nc, _pd(pos), _pd(kpos), _pd(erg_eff), gs.size - 1,
                                    gs.ctypes.data_as(C.POINTER(C.c_int64)), _pd(out))
    return out


def event_weight(p, x, k_init, vifty, max_r, rho_dm=0.45, mcmc_weight=6.0):
    """sln_prob of sampled conversion points (MainRunner.jl:498-557); x, k_init, vifty SoA 3n.
    Returns dict cos_w, jacobian_GR, sln_prob, erg_inf_ini, vel_eng (n each)."""
    x, k_init, vifty = _arr(x).reshape(-1), _arr(k_init).reshape(-1), _arr(vifty).reshape(-1)
    n = x.size // 3
    out = np.zeros(5 * n)
    lib().oracle_event_weight(C.byref(p), n, _pd(x), _pd(k_init), _pd(vifty), float(max_r), float(rho_dm),
                              float(mcmc_weight), _pd(out))
    o = out.reshape(5, n)
    return {k: o[i].copy() for i, k in enumerate(("cos_w", "jacobian_GR", "sln_prob", "erg_inf_ini", "vel_eng"))}


def propagate(p, x0, k0, erg, dw, ln_t0, species, max_crossings=-1, cap=1, nthreads=None):
    """Batched RT.propagate; x0/k0 are SoA (3n) or (n,3) arrays. Returns a dict."""
    x0, k0 = np.asarray(x0, np.float64), np.asarray(k0, np.float64)
    n = np.asarray(erg).size
    if x0.ndim == 2 and x0.shape == (n, 3):
        x0, k0 = x0.T.copy().reshape(-1), k0.T.copy().reshape(-1)
    x0, k0 = _arr(x0), _arr(k0)
    erg = np.broadcast_to(np.asarray(erg, np.float64), (n,)).copy()
    dw = np.broadcast_to(np.asarray(dw, np.float64), (n,)).copy()
    ln_t0 = np.broadcast_to(np.asarray(ln_t0, np.float64), (n,)).copy()
    species = np.broadcast_to(np.asarray(species, np.int8), (n,)).copy()
    out = {k: np.zeros(3 * n) for k in ("x_end", "k_end")}
    out.update({k: np.zeros(n) for k in ("u7_end", "tau_end")})
    out.update({k: np.zeros(n, np.int32) for k in ("status", "n_accept", "n_reject", "n_cross")})
    out.update({k: np.zeros(3 * cap * n) for k in ("xc_pos", "xc_k")})
    out.update({k: np.zeros(cap * n) for k in ("xc_t", "xc_dw", "xc_p")})
    i32p = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))  # noqa: E731
    lib().oracle_propagate(
        C.byref(p), n, _pd(x0), _pd(k0), _pd(erg), _pd(dw), _pd(ln_t0), species.ctypes.data_as(C.POINTER(C.c_int8)),
        max_crossings, _pd(out["x_end"]), _pd(out["k_end"]), _pd(out["u7_end"]), _pd(out["tau_end"]),
        i32p(out["status"]), i32p(out["n_accept"]), i32p(out["n_reject"]), cap, i32p(out["n_cross"]),
        _pd(out["xc_pos"]), _pd(out["xc_k"]), _pd(out["xc_t"]), _pd(out["xc_dw"]), _pd(out["xc_p"]),
        nthreads or os.cpu_count() or 1)
    return out


def sample(p, max_r, seed, ray_offset, n, nthreads=None):
    """find_samples_new + k_norm_Cart: one accepted conversion point per ray (SoA outputs)."""
    out = {"x": np.zeros(3 * n), "k_init": np.zeros(3 * n), "erg": np.zeros(n), "vifty": np.zeros(3 * n),
           "weights": np.zeros(n, np.int32), "attempts": np.zeros(n, np.int32)}
    i32p = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))  # noqa: E731
    lib().oracle_sample(C.byref(p), max_r, seed, ray_offset, n, _pd(out["x"]), _pd(out["k_init"]), _pd(out["erg"]),
                        _pd(out["vifty"]), i32p(out["weights"]), i32p(out["attempts"]),
                        nthreads or os.cpu_count() or 1)
    return out


def sampler_condition(p, x, vloc, E):
    return lib().oracle_sampler_condition(C.byref(p), _pd(_arr(x)), _pd(_arr(vloc)), E)
