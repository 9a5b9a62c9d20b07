#!/bin/bash
# Dev: tail donation -- bit-identity on 20k rays of three configurations, then bench.py on
# the pipelined small-batch shapes and the single-stream headline for several lane counts.
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 tools/exp_donate.py > gpurun_out/donate_id.log 2>&1 || exit 1
for cfg in "1000000 3 0" "1000000 3 8" "1000000 3 16" "1000000 3 32" "1250000 3 0" "1250000 3 16" "10000000 1 0" "10000000 1 16" "1000000 1 0" "1000000 1 16"; do
  read -r rays st dn <<< "$cfg"
  timeout -k 10 300 python3 bench.py --rays $rays --streams $st --donate $dn --steps 10 --warmup 2 --no-cpu-baseline --no-pcie 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print($rays, $st, $dn, d['value'], d['roofline']['kernel_ms'])" || exit 1
done
