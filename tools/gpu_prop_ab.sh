#!/bin/bash
# Dev: propagate outputs of the current build against tools/build/libart_base.so (bit-identical?),
# then interleaved kernel timings of both on the 1e7-ray flat batch.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ART_LIB=${AB_BASE:-tools/build/libart_base.so} timeout -k 10 300 python3 tools/exp_prop_ab.py /tmp/prop_base.npz > gpurun_out/prop_base.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/exp_prop_ab.py /tmp/prop_new.npz > gpurun_out/prop_new.log 2>&1 || exit $?
python3 - <<'PY'
import numpy as np
a, b = np.load("/tmp/prop_base.npz"), np.load("/tmp/prop_new.npz")
bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
print("propagate identical" if not bad else f"propagate DIFFER: {bad}")
PY
REPS=${REPS:-3} bash tools/ab_multi.sh ${AB_BASE:-tools/build/libart_base.so} adiabatic_raytracer_amd/lib/libart.so
