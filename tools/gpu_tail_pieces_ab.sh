#!/bin/bash
# Dev: the last ART_HOST_TAIL_PIECES pieces of a streamed call finalized on the integrator's CUs
# after it ends (0: all on the helper CUs). Usage: tools/gpu_tail_pieces_ab.sh TAG LIB
TAG=$1; LIB=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/${TAG}_tail_pieces.jsonl
for rep in 1 2; do for t in 0 1 2 3; do
  echo "== tail pieces $t" >> $O
  ART_LIB=$LIB ART_HOST_TAIL_PIECES=$t timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream >> $O 2>> gpurun_out/${TAG}.err || exit 1
done; done
echo "== tail pieces 2, then the single launch (bit-identical check)" >> $O
ART_LIB=$LIB ART_HOST_TAIL_PIECES=2 timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream single >> $O 2>> gpurun_out/${TAG}.err || exit 1
echo done
