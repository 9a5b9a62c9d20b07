#!/bin/bash
# A/B of small-batch builds: the GR configs[3] tail ray alone and the flat 1e6 batch's longest ray
# alone (tools/exp_gr_tail.py), interleaved: usage gpu_small_ab.sh lib1.so lib2.so ...
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2 3; do
  for lib in "$@"; do
    echo "$lib gr $(ART_LIB=$lib timeout -k 10 120 python3 tools/exp_gr_tail.py 1 717277 2>/dev/null | tail -1 | cut -c1-130)" || exit 1
    echo "$lib flat $(ART_LIB=$lib TAIL_KW='{"theta_m": 0.2, "mass_a": 1e-5, "flat": true}' timeout -k 10 120 python3 tools/exp_gr_tail.py 1000000 2>/dev/null | tail -1 | cut -c1-130)" || exit 1
  done
done
