#!/bin/bash
# Interleaved A/B of libart builds on configs[3]'s longest ray (717277) alone on the one-wave-per-ray
# tail kernel (tools/exp_gr_tail.py, TAIL_DONATE=4): µs per attempt, one process per run.
# Usage: ROUNDS=3 bash tools/ab_tail.sh OUT.jsonl LIB [LIB ...]   (LIB "base" = adiabatic_raytracer_amd/lib/libart.so)
OUT=$1; shift
ROUNDS=${ROUNDS:-3}
for r in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    if [ "$lib" = base ]; then
      line=$(TAIL_DONATE=4 timeout -k 10 200 python3 -u tools/exp_gr_tail.py 1000000 717277 2>/dev/null | tail -1) || exit 1
    else
      line=$(ART_LIB=$lib TAIL_DONATE=4 timeout -k 10 200 python3 -u tools/exp_gr_tail.py 1000000 717277 2>/dev/null | tail -1) || exit 1
    fi
    echo "{\"round\": $r, \"lib\": \"$lib\", \"result\": $line}" >> "$OUT"
  done
done
