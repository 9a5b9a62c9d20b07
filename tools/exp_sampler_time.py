"""Dev: sample_kernel time (HIP events via torch) for the 1e7-ray flat forward roots and for
the 32-point scan's slowest-to-sample point (m_a = 1e-6, B0 = 2e14, P = 0.5 s: maxR 342 km)."""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402
from adiabatic_raytracer_amd.scan import scan_grid  # noqa: E402

cases = [("flat1e7", dict(theta_m=0.2, mass_a=1e-5, flat=True), 10_000_000)]
big = max(scan_grid(), key=lambda g: A.Params(**g).max_r())
cases.append(("scan_maxR_point_1e6", big, 1_000_000))
for name, kw, n in cases:
    eng = Engine(A.Params(**kw))
    eng.forward_roots(min(n, 100000), seed=1769)  # warm-up
    ms = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        inp = eng.forward_roots(n, seed=1769)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    s = inp["sample"]
    print(json.dumps({"case": name, "rays": n, "max_r": A.Params(**kw).max_r(), "ms": ms,
                      "attempts_mean": float(s["attempts"].double().mean()),
                      "x_sum": float(s["x"].double().sum()), "weights_sum": int(s["weights"].sum()),
                      # every sampled array, bit for bit
                      "sha": hashlib.sha256(b"".join(v.contiguous().cpu().numpy().tobytes()
                                                     for _, v in sorted(s.items()) if torch.is_tensor(v))
                                            ).hexdigest()[:16],
                      "keys": sorted(k for k, v in s.items() if torch.is_tensor(v))}), flush=True)
