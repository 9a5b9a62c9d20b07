#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
ART_LIB=${AB_BASE:-tools/build/libart_base.so} timeout -k 10 120 python3 tools/exp_pointwise_ab.py /tmp/pw_base.npz || exit $?
timeout -k 10 120 python3 tools/exp_pointwise_ab.py /tmp/pw_new.npz || exit $?
python3 - <<'PY'
import numpy as np
a, b = np.load("/tmp/pw_base.npz"), np.load("/tmp/pw_new.npz")
for k in a.files:
    d = ~((a[k] == b[k]) | (np.isnan(a[k]) & np.isnan(b[k])))
    print(k, "identical" if not d.any() else f"{int(d.sum())} of {d.size} differ, max rel {np.nanmax(np.abs(a[k][d]-b[k][d])/np.abs(a[k][d]))}")
PY
