# Early graduation beyond the one batch: configs[3]'s full bench line (host path, device one
# batch, 16 in flight) and the configs[4] 32-point scan (8 streams), default against ART_HOT_AT=0.
set -o pipefail
for hot in 128 0; do
  ART_HOT_AT=$hot timeout -k 10 400 python3 -u bench.py --config gr --rays 1000000 --steps 3 --warmup 1 --no-cpu-baseline > ${OUT}_bench_gr_$hot.json 2>/dev/null || exit 1
  ART_HOT_AT=$hot timeout -k 10 300 python3 -u tools/exp_scan_streams.py 1000000 8 32 16 > ${OUT}_scan_$hot.jsonl 2>/dev/null || exit 1
done
