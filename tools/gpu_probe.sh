#!/bin/bash
# Dev: stream probes (tools/probe_streams.hip, tools/probe_cumask.hip)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 8 16; do
  timeout -k 10 60 tools/build/probe_cumask $r >> gpurun_out/probe_cumask.jsonl 2>&1 || exit 1
done
echo done
