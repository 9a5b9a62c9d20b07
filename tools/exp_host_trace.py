# Experiment: the streamed host pipeline's timeline (ART_HOST_TRACE) on the 10^7-ray headline batch, after three untraced calls.
import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch, ctypes as C
import adiabatic_raytracer_amd as A
from adiabatic_raytracer_amd import Engine
eng = Engine(A.Params(theta_m=0.2, mass_a=1e-5, flat=True))
n = 10_000_000
inp = eng.forward_roots(n, seed=1769)
args = [inp[k].cpu().numpy() for k in ("x0", "k0", "erg", "dw", "ln_t0", "species")]
for i in range(4):
    if i == 3:
        os.environ["ART_HOST_TRACE"] = "1"
    t = time.perf_counter()
    out = A.propagate_batch(eng.params, *args, max_crossings=-1)
    print("call", i, (time.perf_counter() - t) * 1e3, "ms", file=sys.stderr, flush=True)
