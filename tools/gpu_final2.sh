#!/bin/bash
# Round-end side figures: GR configs[3] batch, 1e6 / 1.25e6 flat batches, the 32-point scan.
TAG=${1:-r02b}
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 bench.py --config gr --rays 1000000 --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/${TAG}_bench_gr1e6.json 2>/dev/null || exit 1
for cfg in "1000000 3" "1250000 0"; do
  read -r rays st <<< "$cfg"
  timeout -k 10 300 python3 bench.py --rays $rays --streams $st --steps 20 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/${TAG}_bench_flat_${rays}.json 2>/dev/null || exit 1
done
timeout -k 10 300 python3 tools/exp_scan_streams.py 1000000 8 > gpurun_out/${TAG}_param_scan_1e6_8streams.jsonl 2>/dev/null || exit 1
timeout -k 10 300 python3 tools/exp_gr_tail.py 1 717277 > gpurun_out/${TAG}_gr_tail.jsonl 2>/dev/null || exit 1
