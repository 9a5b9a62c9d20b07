"""Dev: the host-pointer path (art_propagate_host, what a Julia ccall runs) on the 1e7-ray flat
batch, for several pipeline settings (ART_HOST_CHUNKS / ART_HOST_SLOTS / ART_HOST_THREADS are
read per call). Prints one JSON line per setting; with ART_HOST_TRACE=1 the library also
prints the host side of every chunk to stderr.
Usage: exp_host_path.py [rays] [setting ...]; a setting is "stream" (the streamed pipeline),
"single", or "chunks,slots" (the chunked pipeline), e.g.
exp_host_path.py 10000000 stream single 4,2"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402
from adiabatic_raytracer_amd._lib import CrossingBuf, SegmentOut, check  # noqa: E402

if os.environ.get("ART_MAPS_OUT"):  # the process's mappings at exit (resolving a crash PC)
    import atexit
    import shutil
    atexit.register(lambda: shutil.copy("/proc/self/maps", os.environ["ART_MAPS_OUT"]))

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
settings = sys.argv[2:] or ["stream", "single"]
eng = Engine(A.Params(theta_m=0.2, mass_a=1e-5, flat=True))
inp = eng.forward_roots(n, seed=1769)
h = {k: inp[k].cpu().numpy() for k in ("x0", "k0", "erg", "dw", "ln_t0", "species")}
lib = A._lib.load()
P = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731


def outputs(fault):
    mk = np.ones if fault else np.zeros
    o = {"x_end": mk(3 * n), "k_end": mk(3 * n), "u7_end": mk(n), "tau_end": mk(n), "status": mk(n, np.int32),
         "n_accept": mk(n, np.int32), "n_reject": mk(n, np.int32), "n_cross": mk(n, np.int32), "xc_pos": mk(3 * n),
         "xc_k": mk(3 * n), "xc_t": mk(n), "xc_dw": mk(n), "xc_p": mk(n)}
    so = SegmentOut(*[P(o[k]) for k in ("x_end", "k_end", "u7_end", "tau_end", "status", "n_accept", "n_reject")])
    xb = CrossingBuf(1, *[P(o[k]) for k in ("n_cross", "xc_pos", "xc_k", "xc_t", "xc_dw", "xc_p")])
    return o, so, xb


cp = eng.cp
ref = None
for setting in settings:
    chunks = slots = 0
    if setting == "stream":
        os.environ["ART_HOST_MODE"] = "stream"
    elif setting == "single":
        os.environ["ART_HOST_MODE"] = "single"
    else:
        chunks, slots = (int(v) for v in setting.split(","))
        os.environ["ART_HOST_MODE"] = "chunked"
        os.environ["ART_HOST_CHUNKS"] = str(chunks)
        os.environ["ART_HOST_SLOTS"] = str(slots)
    for fault in (True, False):
        times = []
        for rep in range(3):
            o, so, xb = outputs(fault)
            t0 = time.perf_counter()
            check(lib.art_propagate_host(C.byref(cp), n, *[P(h[k]) for k in ("x0", "k0", "erg", "dw", "ln_t0", "species")],
                                         -1, C.byref(so), C.byref(xb)))
            times.append(time.perf_counter() - t0)
        acc = int(o["n_accept"].sum())
        if ref is None:
            ref = o
        same = all(np.array_equal(o[k], ref[k], equal_nan=True) for k in o)
        ms = min(times[1:]) * 1e3
        print(json.dumps({"rays": n, "setting": setting, "chunks": chunks, "slots": slots, "outputs_prefaulted": fault, "ms": ms,
                          "ms_all": [t * 1e3 for t in times], "ray_steps_per_s": acc / (ms * 1e-3),
                          "kernel_ms_sum": lib.art_last_kernel_ms(), "bit_identical_to_first": same}), flush=True)
