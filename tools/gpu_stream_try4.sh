#!/bin/bash
# Dev: the single launch on a CU-masked stream (R = 1, 8) against the plain stream
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 0 1 8; do
  ART_DEV_SINGLE_MASKED=$r timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 single | sed "s|^|masked$r |" >> gpurun_out/${1}_masked.txt 2>> gpurun_out/${1}.err || exit 1
done
echo done
