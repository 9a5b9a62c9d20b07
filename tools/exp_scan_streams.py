"""Dev: the 32-point parameter scan (configs[4]) on one GPU, all points on S streams in flight
(scan.run_points), 1e6 rays each by default. Prints one JSON line per point and a summary."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from adiabatic_raytracer_amd.scan import run_points, scan_grid  # noqa: E402

rays = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
streams = int(sys.argv[2]) if len(sys.argv) > 2 else 16
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < min(16, max(4, streams)):
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(16, max(4, streams)))
npts = int(sys.argv[3]) if len(sys.argv) > 3 else 32
donate = int(sys.argv[4]) if len(sys.argv) > 4 else 0
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 1  # (> 1: the later runs reuse the caching allocator's blocks)
for _ in range(reps - 1):
    print(json.dumps(run_points(scan_grid()[:npts], rays, streams=streams, donate=donate)[1] | {"warm-up": True}), flush=True)
recs, summ = run_points(scan_grid()[:npts], rays, streams=streams, donate=donate)
for i, r in enumerate(recs):
    print(json.dumps({k: r.get(k) for k in ("mass_a", "B0", "omega_pul", "kernel_ms", "accepted", "attempts")} | {"point": i}))
print(json.dumps(summ), flush=True)
