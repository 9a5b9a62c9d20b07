#!/bin/bash
# Dev: bench.py at 1e6 rays (1 and 3 streams) and 1e7 for the current build and the given
# library variants, interleaved twice.
cd "$GRAFT_REPO_ROOT" || exit 1
LIBS=(adiabatic_raytracer_amd/lib/libart.so "$@")
for r in 1 2; do
  for lib in "${LIBS[@]}"; do
    for cfg in "1000000 1" "1000000 3" "10000000 1"; do
      read -r rays st <<< "$cfg"
      ART_LIB=$lib timeout -k 10 200 python3 bench.py --rays $rays --streams $st --steps 10 --warmup 2 --no-cpu-baseline --no-pcie 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$lib', $rays, $st, d['value'])" || exit 1
    done
  done
done
