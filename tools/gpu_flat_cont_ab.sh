#!/bin/bash
# A/B of continuation builds on the 8-GPU shard size (1.25e6 flat rays, 3 passes in flight,
# tail donation 16) and 1e6 rays: usage gpu_flat_cont_ab.sh lib1.so lib2.so ...
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2 3; do
  for lib in "$@"; do
    for rays in 1250000 1000000; do
      ART_LIB=$lib timeout -k 10 200 python3 bench.py --rays $rays --steps 20 --warmup 2 --no-cpu-baseline --no-pcie 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$lib', $rays, '%.4e' % d['value'], round(d['ms_per_step'], 3))" || exit 1
    done
  done
done
