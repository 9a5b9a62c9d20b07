"""Dev experiment (run under rocprofv3 --pmc): one propagate launch of 1e6 flat rays at
interp_points 50 (the reference's) and 2 (no interior scan points), so the PMC rows of the
two propagate_kernel dispatches split the dynamic instruction counts between the resonance
scan and the rest. Prints the launches' statistics as JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
for ip in (50, 2):
    eng = Engine(A.Params(theta_m=0.2, mass_a=1e-5, flat=True, interp_points=ip))
    inp = eng.forward_roots(n, seed=1769)
    out = eng.alloc_out(n)
    eng.propagate(inp, out)
    ms = eng.kernel_ms()
    print(json.dumps({"interp_points": ip, "kernel_ms": ms, **A.raytracer.last_stats()}), flush=True)
    torch.cuda.synchronize()
