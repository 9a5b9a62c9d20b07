#!/bin/bash
# Interleaved A/B of libart builds on bench.py's host path (the streamed pipeline, 1e7 flat rays):
# one process per run so each loads its own library; one JSON line per run.
# Usage: ROUNDS=3 STEPS=10 bash tools/ab_bench.sh OUT.jsonl LIB [LIB ...]   ("base" = the in-tree libart.so)
OUT=$1; shift
ROUNDS=${ROUNDS:-3}
STEPS=${STEPS:-10}
EXTRA=${EXTRA:-}
for r in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    if [ "$lib" = base ]; then
      line=$(timeout -k 10 300 python3 -u bench.py --steps "$STEPS" --warmup 2 --no-device --no-cpu-baseline $EXTRA 2>/dev/null | tail -1) || exit 1
    else
      line=$(ART_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps "$STEPS" --warmup 2 --no-device --no-cpu-baseline $EXTRA 2>/dev/null | tail -1) || exit 1
    fi
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'round': $r, 'lib': '$lib', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms'], 'span_ms': d['roofline']['kernel_span_ms']}))" "$line" >> "$OUT"
  done
done
