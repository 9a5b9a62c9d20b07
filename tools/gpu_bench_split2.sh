#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in "10000000 1" "10000000 2" "10000000 3" "1250000 4" "10000000 1" "10000000 2"; do
  read -r rays st <<< "$cfg"
  timeout -k 10 300 python3 bench.py --rays $rays --streams $st --steps 10 --warmup 2 --no-cpu-baseline --no-pcie 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print($rays, $st, d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['achieved_wall'])" || exit 1
done
