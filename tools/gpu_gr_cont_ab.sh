#!/bin/bash
# A/B of GR continuation builds on the configs[3] bench line (1e6 GR rays, 3 passes in flight,
# tail donation 16): usage gpu_gr_cont_ab.sh lib1.so lib2.so ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2 3; do
  for lib in "$@"; do
    ART_LIB=$lib timeout -k 10 200 python3 bench.py --config gr --rays 1000000 --steps 5 --warmup 1 --no-cpu-baseline --no-pcie 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$lib', '%.4e' % d['value'], round(d['ms_per_step'], 2), d['kernel_stats']['accepted'])" || exit 1
  done
done
