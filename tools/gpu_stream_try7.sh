#!/bin/bash
# Dev: which CUs to reserve for the streamed pipeline's helpers (local index per XCD)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for loc in 0 16 31; do
  ART_HOST_RESERVE_LOCAL=$loc timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream | sed "s|^|loc$loc |" >> gpurun_out/${1}.txt 2>> gpurun_out/${1}.err || exit 1
  ART_HOST_RESERVE_LOCAL=$loc ART_DEV_SINGLE_MASKED=8 timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 single | sed "s|^|loc$loc-masked |" >> gpurun_out/${1}.txt 2>> gpurun_out/${1}.err || exit 1
done
echo done
