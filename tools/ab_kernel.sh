#!/bin/bash
# Interleaved A/B of libart builds on the device-resident 1e7-ray flat batch (tools/exp_sections.py:
# the integrator's HIP-event time), one process per run so each loads its own library.
# Usage: ROUNDS=3 bash tools/ab_kernel.sh OUT.jsonl LIB [LIB ...]   (LIB "base" = adiabatic_raytracer_amd/lib/libart.so)
OUT=$1; shift
ROUNDS=${ROUNDS:-3}
for r in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    if [ "$lib" = base ]; then
      line=$(timeout -k 10 200 python3 -u tools/exp_sections.py 2>/dev/null | tail -1) || exit 1
    else
      line=$(ART_LIB=$lib timeout -k 10 200 python3 -u tools/exp_sections.py 2>/dev/null | tail -1) || exit 1
    fi
    echo "{\"round\": $r, \"lib\": \"$lib\", \"result\": $line}" >> "$OUT"
  done
done
