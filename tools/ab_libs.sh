#!/bin/bash
# Interleaved A/B of several libart.so builds: the 1e7-ray flat bulk (kernel ms, best of the
# timed launches) and the GR configs[3] tail ray 717277 alone (µs per attempt), REPS rounds.
# usage: REPS=3 ab_libs.sh lib1.so lib2.so ...   -> gpurun_out/ab_libs.log + summary
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
REPS=${REPS:-3}
for r in $(seq 1 "$REPS"); do
  for lib in "$@"; do
    ART_LIB=$lib timeout -k 10 120 python3 tools/ab.py 10000000 flat >> gpurun_out/ab_libs.log 2>/dev/null || exit $?
    if [ -z "$NO_GR" ]; then
      echo "{\"lib\": \"$lib\", \"gr_tail\": $(ART_LIB=$lib timeout -k 10 120 python3 tools/exp_gr_tail.py 1 717277 2>/dev/null | tail -1)}" >> gpurun_out/ab_libs.log || exit $?
    fi
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list); g = collections.defaultdict(list)
for l in open("gpurun_out/ab_libs.log"):
    if not l.startswith("{"): continue
    j = json.loads(l)
    if "kernel_ms" in j: d[j["lib"]].append((j["kernel_ms"], j["accepted"], j["scan_evals"]))
    elif isinstance(j.get("gr_tail"), dict): g[j["lib"]].append(j["gr_tail"])
for k, v in d.items():
    ms = [x[0] for x in v]
    gt = g.get(k, [])
    gts = [x.get("us_per_attempt", x) for x in gt]
    print(f"{k:45s} flat min {min(ms):7.2f} ms  all {' '.join(f'{x:.2f}' for x in ms)}  acc {v[0][1]} scan {v[0][2]}  gr {gts}")
PY
