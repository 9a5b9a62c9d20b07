#!/bin/bash
# Dev: the sampler of the current build (or NEW=lib.so) against a saved baseline build (tools/build/libart_base.so):
# bit-identical samples on three configurations and the wall time of each.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=${N:-200000}
ART_LIB=tools/build/libart_base.so timeout -k 10 200 python3 tools/exp_sampler_ab.py /tmp/samp_base.npz $N > gpurun_out/samp_base.log 2>&1 || exit $?
ART_LIB=${NEW:-adiabatic_raytracer_amd/lib/libart.so} timeout -k 10 200 python3 tools/exp_sampler_ab.py /tmp/samp_new.npz $N > gpurun_out/samp_new.log 2>&1 || exit $?
python3 - <<'PY'
import numpy as np
a, b = np.load("/tmp/samp_base.npz"), np.load("/tmp/samp_new.npz")
bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
print("identical" if not bad else f"DIFFER: {bad}")
for k in bad:
    d = a[k] != b[k]
    print(k, int(d.sum()), "of", d.size)
PY
