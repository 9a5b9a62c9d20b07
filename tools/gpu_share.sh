#!/bin/bash
# Dev: persistent-grid share (ART_GRID_SHARE) against streams in flight on the 1e6 batch.
cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in "1.0 3" "0.97 3" "0.94 3" "0.9 3" "0.97 2" "0.94 2"; do
  read -r sh st <<< "$cfg"
  ART_GRID_SHARE=$sh timeout -k 10 200 python3 bench.py --rays 1000000 --streams $st --steps 20 --warmup 2 --no-cpu-baseline --no-pcie 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('share $sh streams $st', d['value'])" || exit 1
done
