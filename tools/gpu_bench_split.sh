#!/bin/bash
# Dev: per-GPU shard sizes of the 8/4/2-GPU strong-scaling split against streams in flight.
cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in "1250000 2" "1250000 3" "2500000 2" "2500000 3" "5000000 1" "5000000 2"; do
  read -r rays st <<< "$cfg"
  timeout -k 10 300 python3 bench.py --rays $rays --streams $st --steps 10 --warmup 2 --no-cpu-baseline --no-pcie 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print($rays, $st, d['value'])" || exit 1
done
