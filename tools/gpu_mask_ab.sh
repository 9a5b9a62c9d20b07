#!/bin/bash
# Dev: what masking 8 CUs (one per XCD) costs the plain integrator, with the grid sized for all
# 256 CUs (512 blocks) and for the 248 the mask leaves (libart_g248.so, -DART_DEV_GRID_CUS=248).
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/${TAG}_mask.jsonl
for rep in 1 2; do
  echo "== unmasked, 512 blocks" >> $O
  timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 single >> $O 2>> gpurun_out/${TAG}.err || exit 1
  echo "== masked 8, 512 blocks" >> $O
  ART_DEV_SINGLE_MASKED=8 timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 single >> $O 2>> gpurun_out/${TAG}.err || exit 1
  echo "== masked 8, 496 blocks" >> $O
  ART_LIB=tools/build/libart_g248.so ART_DEV_SINGLE_MASKED=8 timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 single >> $O 2>> gpurun_out/${TAG}.err || exit 1
done
echo done
