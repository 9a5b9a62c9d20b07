#!/bin/bash
# Interleaved A/B of several builds of libart.so on the 1e7-ray flat batch (the bench
# workload), each timed in its own process, REPS rounds: usage ab_multi.sh lib1.so lib2.so ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
REPS=${REPS:-3}
N=${AB_N:-10000000}
for r in $(seq 1 "$REPS"); do
  for lib in "$@"; do
    ART_LIB=$lib timeout -k 10 120 python3 tools/ab.py "$N" flat >> gpurun_out/ab_multi.log 2>/dev/null || exit $?
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ab_multi.log"):
    if l.startswith("{"):
        j = json.loads(l); d[j["lib"]].append(j["kernel_ms"])
for k, v in d.items():
    print(f"{k:50s} min {min(v):8.3f} ms  all {' '.join(f'{x:.2f}' for x in v)}")
PY
