#!/bin/bash
# Dev: the streamed integrator with every piece initialised before it starts
# (ART_HOST_STREAM_SERIAL=1: no input gating) against the normal streamed call.
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/${TAG}_serial.jsonl
for rep in 1 2; do
  echo "== streamed" >> $O
  timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream >> $O 2>> gpurun_out/${TAG}.err || exit 1
  echo "== streamed, inputs all initialised first" >> $O
  ART_HOST_STREAM_SERIAL=1 timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream >> $O 2>> gpurun_out/${TAG}.err || exit 1
done
echo done
