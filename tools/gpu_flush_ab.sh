#!/bin/bash
# Dev A/B: the streamed host pipeline's count-flush interval (ART_STREAM_FLUSH builds from
# `python -m adiabatic_raytracer_amd.build --variant`). Usage: tools/gpu_flush_ab.sh TAG lib1.so ...
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do for lib in adiabatic_raytracer_amd/lib/libart.so "$@"; do
  echo "== $lib" >> gpurun_out/${TAG}_flush.jsonl
  ART_LIB=$lib timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream >> gpurun_out/${TAG}_flush.jsonl 2>> gpurun_out/${TAG}.err || exit 1
done; done
echo done
