"""Experiment (DESIGN §10, configs[3] in one batch): the 10^6-ray GR batch's forward roots from
the GPU sampler, then tools/exp_gr_predict.cpp (the same-algorithm CPU loop with probes) on the
host cores: per ray the attempt count and its ln t and r at attempts 32..4096. Writes
gpurun_out/gr_predict.npz (rays past 128 attempts only)."""
import ctypes as C
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, HERE)
import cpu_same  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 1000000
THREADS = int(os.environ.get("THREADS", "16"))
CFG = {"gr": dict(theta_m=0.0, mass_a=1e-6, flat=False), "flat": dict(theta_m=0.2, mass_a=1e-5, flat=True)}[
    os.environ.get("CONFIG", "gr")]  # (bench.py's configs; CONFIG=flat: the headline's)
TAG = "" if os.environ.get("CONFIG", "gr") == "gr" else "_" + os.environ["CONFIG"]
LIB = os.path.join(HERE, "build", "libexp_gr_predict.so")

if __name__ == "__main__":
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(HERE, "exp_gr_predict.cpp")):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", *cpu_same.FLAGS, os.path.join(HERE, "exp_gr_predict.cpp"), "-o", LIB],
                       check=True)
    if "--build" in sys.argv:
        sys.exit(0)
    import adiabatic_raytracer_amd as A
    from adiabatic_raytracer_amd import Engine
    import oracle as O
    eng = Engine(A.Params(**CFG))
    inp = eng.forward_roots(N, seed=1769)
    x0 = inp["x0"].cpu().numpy()
    k0 = inp["k0"].cpu().numpy()
    erg = inp["erg"].cpu().numpy()
    lib = C.CDLL(LIB)
    cpu_same._lib = lib
    probe = np.full((N, 9, 2), np.nan, np.float32)
    lib.exp_set_probe(probe.ctypes.data_as(C.c_void_p))
    p = O.make_params(**CFG)
    t = time.time()
    r = cpu_same.propagate(p, x0, k0, erg, -1.0, -30.0, 1, max_crossings=-1, nthreads=THREADS)
    print("cpu", time.time() - t, flush=True)
    att = r["n_accept"] + r["n_reject"]
    keep = np.nonzero(att > 128)[0]
    np.savez_compressed(f"gpurun_out/gr_predict_all{TAG}.npz", att=att.astype(np.int32), dt0=probe[:, 8, 0], r0=probe[:, 8, 1])
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed(f"gpurun_out/gr_predict{TAG}.npz", ray=keep, att=att[keep], status=r["status"][keep],
                        tau_end=r["tau_end"][keep], probe=probe[keep], att_hist=np.bincount(np.minimum(att, 100000)))
    print("rays past 128 attempts", keep.size, "max", att.max(), "argmax", att.argmax(), flush=True)
