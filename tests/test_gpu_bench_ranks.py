"""Rehearsal of the driver's N-GPU bench on the one card of a GPU box: bench.py launched by
torch.distributed.run exactly as the SCALE run launches it, here with 8
ranks, every rank on device 0 and gloo for the all-reduce (ART_BENCH_DEVICE /
ART_BENCH_BACKEND). Checks the contract's one JSON line, totals equal to the sum over the
shards (= the single-process run's) and a reduced flux equal to the single-process run's,
bin for bin (Gen_Samples.jl:195-239 merges per-process runs; here one all-reduce). This
makes no scaling claim: the 8 ranks share one GPU."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--rays", "1250000", "--steps", "2", "--warmup", "1", "--no-device", "--no-cpu-baseline"]


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_eight_gloo_ranks_on_one_card():
    env = dict(os.environ, ART_BENCH_DEVICE="0", ART_BENCH_BACKEND="gloo")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "8", *ARGS]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout[-4000:]  # rank 0 only
    multi = lines[0]
    one = _json_lines(subprocess.run([sys.executable, "bench.py", *ARGS], cwd=ROOT, env=dict(os.environ),
                                     capture_output=True, text=True, timeout=300, check=True).stdout)
    assert len(one) == 1
    one = one[0]
    assert multi["n_gpus"] == 8 and one["n_gpus"] == 1
    assert multi["totals"] == one["totals"] and multi["totals"]["rays"] == 1250000
    assert multi["flux_hist"] == one["flux_hist"] and sum(one["flux_hist"]) > 0
    assert multi["value"] > 0 and multi["steps"] == 2 and multi["warmup"] == 1
