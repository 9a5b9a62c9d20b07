"""CPU BASELINE ONLY: builds and loads tools/build/libcpusame.so (tools/cpu_same.cpp), the
engine's algorithm (art_core.h physics, scalar Vern6 + certified scan) on the host cores with
OpenMP, for bench.py's cpu_baseline leg. The product never loads this."""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "cpu_same.cpp")
LIB = os.path.join(HERE, "build", "libcpusame.so")
DEPS = [SRC, os.path.join(HERE, "..", "adiabatic_raytracer_amd", "csrc", "art_core.h"),
        os.path.join(HERE, "..", "include", "art.h")]
# host-only compile of the HIP header with clang (art_core.h's __host__ __device__ functions);
# -march=x86-64-v3: the library also runs on the GPU box's host CPU (AVX2 + FMA)
FLAGS = ["-x", "hip", "--cuda-host-only", "-O3", "-march=x86-64-v3", "-ffp-contract=fast", "-fopenmp", "-std=c++17",
         "-fPIC", "-shared"]
_lib = None


def build():
    if os.path.exists(LIB) and all(os.path.getmtime(LIB) >= os.path.getmtime(d) for d in DEPS):
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, SRC, "-o", LIB + ".tmp"], check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
    return _lib


def propagate(p, x0, k0, erg, dw=-1.0, ln_t0=-30.0, species=1, max_crossings=-1, nthreads=1):
    """p: an oracle.ArtParams (the art_params layout). SoA inputs; returns a dict like
    oracle.propagate's (crossing capacity 1)."""
    n = np.asarray(erg).size
    f64 = lambda a: np.ascontiguousarray(np.broadcast_to(np.asarray(a, np.float64), (n,)))  # noqa: E731
    x0, k0 = np.ascontiguousarray(x0, np.float64).reshape(-1), np.ascontiguousarray(k0, np.float64).reshape(-1)
    erg, dw, ln_t0 = f64(erg), f64(dw), f64(ln_t0)
    sp = np.ascontiguousarray(np.broadcast_to(np.asarray(species, np.int8), (n,)))
    out = {k: np.zeros(3 * n) for k in ("x_end", "k_end", "xc_pos", "xc_k")}
    out.update({k: np.zeros(n) for k in ("u7_end", "tau_end", "xc_t", "xc_dw", "xc_p")})
    out.update({k: np.zeros(n, np.int32) for k in ("status", "n_accept", "n_reject", "n_cross")})
    P = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    lib().cpu_same_propagate(C.byref(p), C.c_int64(n), P(x0), P(k0), P(erg), P(dw), P(ln_t0), P(sp),
                             C.c_int32(max_crossings), *[P(out[k]) for k in (
                                 "x_end", "k_end", "u7_end", "tau_end", "status", "n_accept", "n_reject", "n_cross",
                                 "xc_pos", "xc_k", "xc_t", "xc_dw", "xc_p")], C.c_int32(nthreads))
    return out
