#!/bin/bash
# Dev: the streamed host pipeline's piece size (ART_HOST_PIECE_SHIFT; default 2^19 rays for 10^7).
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/${TAG}_piece.jsonl
for rep in 1 2; do for sh in 0 18 17 20; do
  echo "== piece shift $sh" >> $O
  ART_HOST_PIECE_SHIFT=$sh timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream >> $O 2>> gpurun_out/${TAG}.err || exit 1
done; done
echo done
