#!/bin/bash
# Dev A/B session: integrator builds (tools/ab_libs.sh: 1e7 flat kernel ms, GR tail ray µs per
# attempt), the sampler of one build against libart_base.so (bit-identical samples, ms per 1e7),
# and the host path's chunk trace. Usage: SAMP=lib.so tools/gpu_ab.sh TAG lib1.so lib2.so ...
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  REPS=${REPS:-3} timeout -k 10 700 bash tools/ab_libs.sh "$@" > gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
fi
if [ -n "$SAMP" ]; then
  NEW=$SAMP timeout -k 10 400 bash tools/gpu_sampler_ab.sh > gpurun_out/${TAG}_sampler_identity.txt 2>&1 || exit 1
  for lib in tools/build/libart_base.so $SAMP; do
    ART_LIB=$lib timeout -k 10 200 python3 -u tools/exp_sampler_time.py >> gpurun_out/${TAG}_sampler_time.jsonl 2>> gpurun_out/${TAG}.err || exit 1
  done
fi
if [ -n "$HOST" ]; then
  ART_HOST_TRACE=1 timeout -k 10 300 python3 -u tools/exp_host_path.py 10000000 8,3 8,2 > gpurun_out/${TAG}_host_path.jsonl 2> gpurun_out/${TAG}_host_path.err || exit 1
fi
echo done
