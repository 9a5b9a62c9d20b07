#!/bin/bash
# Dev: shard size x streams in flight with tail donation (auto 16 lanes when streams > 1).
cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in "1000000 2" "1000000 3" "1000000 4" "1250000 2" "1250000 3" "1250000 4" "2500000 2" "2500000 3" "5000000 2" "5000000 3" "10000000 2"; do
  read -r rays st <<< "$cfg"
  timeout -k 10 300 python3 bench.py --rays $rays --streams $st --steps 10 --warmup 2 --no-cpu-baseline --no-pcie 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print($rays, $st, d['config']['tail_donation'], d['value'])" || exit 1
done
