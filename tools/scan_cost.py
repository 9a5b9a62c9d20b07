"""Dev experiment: propagate-kernel time on 1e6 flat rays vs ContinuousCallback interp_points
(the resonance-scan density). Prints one JSON line per setting."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
for ip in (50, 26, 2):
    eng = Engine(A.Params(theta_m=0.2, mass_a=1e-5, flat=True, interp_points=ip))
    inp = eng.forward_roots(n, seed=1769)
    out = eng.alloc_out(n)
    for _ in range(2):
        eng.propagate(inp, out)
        ms = eng.kernel_ms()
    st = A.raytracer.last_stats()
    print(json.dumps({"interp_points": ip, "kernel_ms": ms, "accepted": st["accepted"], "scan_evals": st["scan_evals"],
                      "ray_steps_per_s": st["accepted"] / ms * 1e3}), flush=True)
    torch.cuda.synchronize()
