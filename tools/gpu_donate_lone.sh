#!/bin/bash
# Dev: the lone 1e7-ray pass with tail donation (two levels, tail kernel) against none, interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  for d in 0 4 16 63; do
    timeout -k 10 300 python3 -u bench.py --steps 5 --donate $d --no-cpu-baseline --no-pcie | sed "s|^|donate$d |" >> gpurun_out/${1}.txt 2>> gpurun_out/${1}.err || exit 1
  done
done
echo done
