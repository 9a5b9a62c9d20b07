# Early graduation (SegOut::hot): the hot-ray bit-exact, tail and longest-ray tests, then an
# interleaved A/B on configs[3] as one 10^6-ray batch (the default against ART_HOT_AT=0). OUT prefix.
set -o pipefail
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tail_donation.py tests/test_longest_ray.py -m gpu > ${OUT}_tests.log 2>&1 || exit 1
for r in 1 2 3; do
  for hot in 128 0; do
    ART_HOT_AT=$hot timeout -k 10 300 python3 -u bench.py --config gr --rays 1000000 --steps 3 --warmup 1 --no-cpu-baseline --no-device 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'hot_at': $hot, 'r': $r, 'value': d['value'], 'ms': d['ms_per_step'], 'kms': d['roofline']['kernel_ms']}))" >> ${OUT}_gr.jsonl || exit 1
  done
done
