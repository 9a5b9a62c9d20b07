#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
for lib in adiabatic_raytracer_amd/lib/libart.so tools/build/libart_w1.so; do
  ART_LIB=$lib timeout -k 10 300 python3 bench.py --config gr --rays 1000000 --streams 1 --steps 2 --warmup 1 --no-cpu-baseline --no-pcie 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$lib gr1e6', d['value'], d['roofline']['kernel_ms'])" || exit 1
  ART_LIB=$lib timeout -k 10 300 python3 bench.py --config gr --rays 4000000 --streams 1 --steps 2 --warmup 1 --no-cpu-baseline --no-pcie 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$lib gr4e6', d['value'], d['roofline']['kernel_ms'])" || exit 1
done
done
