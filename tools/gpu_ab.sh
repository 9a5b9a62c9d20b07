#!/bin/bash
# GPU session: the GPU test suite, A/B kernel timings of libart.so against a reference
# build (ART_LIB_PREV, when set) on 1e6-ray flat/GR batches, and the
# default bench line. Every GPU step has its own time limit; the chain stops at the first
# step that crashes or times out (ordinary pytest failures, rc 1, do not stop it).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 tools/ab.py > gpurun_out/ab_new.log 2>&1 || exit $?
if [ -n "$ART_LIB_PREV" ] && [ -f "$ART_LIB_PREV" ]; then  # a build with the same C ABI
  ART_LIB=$ART_LIB_PREV timeout -k 10 200 python3 tools/ab.py > gpurun_out/ab_prev.log 2>&1 || exit $?
fi
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
exit 0
