#!/bin/bash
# Dev: wave priority for outlier rays (ART_PRIO_ITERS) on and off: the 32-point scan wall, the
# GR 1e6 batch and the flat 1e7 kernel.
cd "$GRAFT_REPO_ROOT" || exit 1
for lib in adiabatic_raytracer_amd/lib/libart.so tools/build/libart_noprio.so; do
  echo "== $lib"
  ART_LIB=$lib timeout -k 10 200 python3 tools/exp_scan_streams.py 1000000 8 2>&1 | tail -1 || exit 1
  ART_LIB=$lib timeout -k 10 200 python3 tools/exp_gr_tail.py 1000000 2>&1 | grep batch_kernel_ms | cut -c1-60 || exit 1
done
REPS=2 bash tools/ab_multi.sh tools/build/libart_noprio.so adiabatic_raytracer_amd/lib/libart.so
