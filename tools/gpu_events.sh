#!/bin/bash
# Dev: event throughput (main_runner_tree) with the small-batch tail mode, forest donation off/on
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for d in 0 16; do
  ART_DONATE=$d timeout -k 10 300 python3 -u tools/exp_events.py gr 1000,10000 0 >> gpurun_out/${1}_events_gr.jsonl 2>> gpurun_out/${1}.err || exit 1
  ART_DONATE=$d timeout -k 10 300 python3 -u tools/exp_events.py flat 1000,10000,100000 0 >> gpurun_out/${1}_events_flat.jsonl 2>> gpurun_out/${1}.err || exit 1
done
echo done
