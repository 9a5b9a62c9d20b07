"""TEST TOOL ONLY: builds and loads tools/build/libcorecheck.so, a host compile of the
product's physics header (art_core.h), so CPU tests can compare the analytic kernels'
math with the oracle without a GPU. The product never loads this."""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "corecheck.cpp")
LIB = os.path.join(HERE, "build", "libcorecheck.so")
DEPS = [SRC, os.path.join(HERE, "..", "adiabatic_raytracer_amd", "csrc", "art_core.h"),
        os.path.join(HERE, "..", "include", "art.h")]
_lib = None
pd = C.POINTER(C.c_double)


def build():
    if os.path.exists(LIB) and all(os.path.getmtime(LIB) >= os.path.getmtime(d) for d in DEPS):
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", SRC, "-o", LIB], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        _lib.cc_condition.restype = C.c_double
        _lib.cc_prob_single.restype = C.c_double
        _lib.cc_sampler_condition.restype = C.c_double
        for n in ("cc_condition", "cc_prob_single", "cc_sampler_condition", "cc_rhs", "cc_hamiltonian",
                  "cc_initial_state", "cc_back_transform"):
            pass
    return _lib


def P(a):
    return np.ascontiguousarray(a, np.float64).ctypes.data_as(pd)


def rhs(p, species, u, tau, erg):
    du = np.zeros(7)
    lib().cc_rhs(C.byref(p), int(species), P(u), C.c_double(tau), C.c_double(erg), P(du))
    return du


def condition(p, u, tau):
    return lib().cc_condition(C.byref(p), P(u), C.c_double(tau))


def hamiltonian(p, x, k, T, E):
    H, gx, gk, gT = np.zeros(1), np.zeros(3), np.zeros(3), np.zeros(1)
    lib().cc_hamiltonian(C.byref(p), P(x), P(k), C.c_double(T), C.c_double(E), P(H), P(gx), P(gk), P(gT))
    return H[0], gx, gk, gT[0]


def initial_state(p, x0, k0, erg, dw):
    u = np.zeros(7)
    lib().cc_initial_state(C.byref(p), P(x0), P(k0), C.c_double(erg), C.c_double(dw), P(u))
    return u


def back_transform(p, u, erg):
    x, k = np.zeros(3), np.zeros(3)
    lib().cc_back_transform(C.byref(p), P(u), C.c_double(erg), P(x), P(k))
    return x, k


def prob_single(p, pos, kpos, erg):
    return lib().cc_prob_single(C.byref(p), P(pos), P(kpos), C.c_double(erg))


def sampler_condition(p, x, vl, E):
    return lib().cc_sampler_condition(C.byref(p), P(x), P(vl), C.c_double(E))


def sampler_signs(p, x, vl, E):
    """(condition, sampler_sign_fast verdict) at each of the n points x (n, 3)"""
    x, vl, E = (np.ascontiguousarray(a, np.float64) for a in (x, vl, E))
    n = len(E)
    cond, sgn = np.zeros(n), np.zeros(n, np.int32)
    lib().cc_sampler_signs(C.byref(p), C.c_int64(n), P(x), P(vl), P(E), P(cond),
                           sgn.ctypes.data_as(C.POINTER(C.c_int32)))
    return cond, sgn


def attempt_uniforms(seed, ray, attempt):
    U = np.zeros(10)
    lib().cc_attempt_uniforms(C.c_uint64(seed), C.c_uint64(ray), C.c_uint32(attempt), P(U))
    return U


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().cc_philox(c, k, o)
    return list(o)


def sincos(x):
    x = np.ascontiguousarray(x, np.float64)
    s, c = np.zeros_like(x), np.zeros_like(x)
    lib().cc_sincos(P(x), C.c_int64(x.size), P(s), P(c))
    return s, c


def walk(cw, nper, st, bits):
    """(found or -1, [ip, last_s, last_j, lc_ok]) of walk_codes_bits (bits) or walk_codes_loop."""
    c = (C.c_uint * 4)(*[int(v) & 0xFFFFFFFF for v in cw])
    s = (C.c_int * 4)(*st)
    r = lib().cc_walk(c, C.c_int(nper), s, C.c_int(1 if bits else 0))
    return r, list(s)


def exp_fma(x):
    x = np.ascontiguousarray(x, np.float64)
    y = np.zeros_like(x)
    lib().cc_exp_fma(P(x), C.c_int64(x.size), P(y))
    return y


def log_fma(x):
    x = np.ascontiguousarray(x, np.float64)
    y = np.zeros_like(x)
    lib().cc_log_fma(P(x), C.c_int64(x.size), P(y))
    return y


def metric_d(r, rs):
    o = np.zeros(4)
    lib().cc_metric_d(C.c_double(r), C.c_double(rs), P(o))
    return o


def certified_code(p, u0, f0, u1, f1, h, tau, two_sided=False):
    return int(lib().cc_certified_code(C.byref(p), P(u0), P(f0), P(u1), P(f1), C.c_double(h), C.c_double(tau),
                                       int(two_sided)))
