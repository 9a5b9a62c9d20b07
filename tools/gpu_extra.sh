#!/bin/bash
# GPU tests, kernel-time split (tools/scan_cost.py), flat/GR timings (tools/ab.py) and a
# 2-rank rehearsal of the N > 1 bench path on one GPU (gloo). Stops at the first GPU step
# that crashes or times out.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 tools/scan_cost.py > gpurun_out/scan_cost.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/ab.py > gpurun_out/ab.log 2>&1 || exit $?
ART_BENCH_DEVICE=0 ART_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 2 --warmup 1 \
  --rays 2000000 --no-cpu-baseline > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || exit $?
exit 0
