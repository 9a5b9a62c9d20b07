"""Dev: where the 32-point scan's sampling time goes (scan.run_points' sample_s): per point the
Engine set-up (host) and sample_kernel's time alone on one stream (HIP events), then the same
dispatch over 8 streams as run_points. One JSON line per point and a summary."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import adiabatic_raytracer_amd as A  # noqa: E402
from adiabatic_raytracer_amd import Engine  # noqa: E402
from adiabatic_raytracer_amd.scan import dispatch, scan_grid  # noqa: E402

rays = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
grid = scan_grid()
torch.cuda.synchronize()
engs, setup = [], []
t0 = time.perf_counter()
for kw in grid:
    t = time.perf_counter()
    p = A.Params(**kw)
    mr = p.max_r()
    engs.append((Engine(p), mr))
    setup.append(time.perf_counter() - t)
t_setup = time.perf_counter() - t0
engs[0][0].forward_roots(10000, seed=1769)  # warm-up
torch.cuda.synchronize()
alone = []
for i, (e, mr) in enumerate(engs):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t = time.perf_counter()
    e0.record()
    e.forward_roots(rays, seed=1769)
    e1.record()
    torch.cuda.synchronize()
    alone.append(e0.elapsed_time(e1))
    print(json.dumps({"point": i, "max_r": mr, "setup_ms": setup[i] * 1e3, "sample_ms": alone[-1],
                      "wall_ms": (time.perf_counter() - t) * 1e3}), flush=True)
ss = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(7)]
live = sorted(range(len(engs)), key=lambda i: -engs[i][1])
t = time.perf_counter()
dispatch(live, lambda i: engs[i][0].forward_roots(rays, seed=1769), ss)
torch.cuda.synchronize()
t_conc = time.perf_counter() - t
# the same dispatch with every output allocated beforehand on its stream's pool (the launches alone)
import ctypes as C  # noqa: E402
from adiabatic_raytracer_amd.engine import _p, _stream  # noqa: E402
pre = {}
t = time.perf_counter()
for q, i in enumerate(live):
    with torch.cuda.stream(ss[q % len(ss)]):
        e = engs[i][0]
        pre[i] = {k: e.empty(3 * rays) for k in ("x", "k_init", "vifty")} | {"erg": e.empty(rays)} | \
            {k: e.empty(rays, dtype=torch.int32) for k in ("weights", "attempts")}
torch.cuda.synchronize()
t_alloc = time.perf_counter() - t


def launch(i):
    e, mr = engs[i]
    o = pre[i]
    rc = e.lib.art_sample_conversion_points_device(C.byref(e.cp), float(mr), 1769, 0, rays,
                                                   *[_p(o[k]) for k in ("x", "k_init", "erg", "vifty", "weights", "attempts")],
                                                   _stream())
    assert rc == 0


t = time.perf_counter()
dispatch(live, launch, ss)
torch.cuda.synchronize()
t_pre = time.perf_counter() - t
print(json.dumps({"setup_s": t_setup, "sum_sample_alone_s": sum(alone) / 1e3, "sample_8streams_s": t_conc,
                  "alloc_s": t_alloc, "sample_8streams_preallocated_s": t_pre}), flush=True)
