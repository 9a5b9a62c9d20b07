#!/bin/bash
# Dev: propagate outputs of the current build against tools/build/libart_base.so (bit-identical?)
# and the GR 1e6 batch (configs[3]) kernel time of both, interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_prop_ab.sh || exit 1
for r in 1 2; do
  for lib in tools/build/libart_base.so adiabatic_raytracer_amd/lib/libart.so; do
    ART_LIB=$lib timeout -k 10 200 python3 tools/exp_gr_tail.py 1000000 2>&1 | grep batch_kernel_ms | cut -c1-60 | sed "s|^|$lib |" || exit 1
  done
done
