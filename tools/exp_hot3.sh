# Early graduation with and without the smallest-initial-step-first claim order (ART_HOT_ORDER),
# and off (ART_HOT_AT=0): configs[3] as one 10^6-ray batch, interleaved; then the tail-donation and
# longest-ray tests. OUT prefix.
set -o pipefail
for r in 1 2 3; do
  for v in "1 128" "0 128" "1 0"; do
    set -- $v
    ART_HOT_ORDER=$1 ART_HOT_AT=$2 timeout -k 10 300 python3 -u bench.py --config gr --rays 1000000 --steps 3 --warmup 1 --no-cpu-baseline --no-device 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'order': $1, 'hot_at': $2, 'r': $r, 'value': d['value'], 'ms': d['ms_per_step'], 'kms': d['roofline']['kernel_ms']}))" >> ${OUT}_gr.jsonl || exit 1
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tail_donation.py tests/test_longest_ray.py tests/test_edges.py -m gpu > ${OUT}_tests.log 2>&1
