#!/bin/bash
# Dev A/B: block-size builds of the integrator, single stream at 1e7 rays (ab_multi) and the
# 1.25e6-ray per-GPU share of an 8-GPU run with 1 and 2 streams (bench.py).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
REPS=2 bash tools/ab_multi.sh adiabatic_raytracer_amd/lib/libart.so tools/build/libart_b128.so tools/build/libart_b64.so > gpurun_out/ab_block_1e7.txt 2>&1 || exit $?
for lib in adiabatic_raytracer_amd/lib/libart.so tools/build/libart_b128.so tools/build/libart_b64.so; do
  for s in 1 2; do
    ART_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pcie --streams $s --rays 1250000 --steps 20 --warmup 3 > gpurun_out/tmp.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/tmp.json').read().strip().splitlines()[-1]); print('$lib', $s, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" >> gpurun_out/ab_block_125.txt
  done
done
