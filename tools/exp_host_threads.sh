# The host copy pool's size (ART_HOST_THREADS, default 7) on the headline host path, interleaved (OUT file).
set -o pipefail
for r in 1 2 3; do
  for t in 7 11 15; do
    line=$(ART_HOST_THREADS=$t timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-device --no-cpu-baseline 2>/dev/null | tail -1) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'round': $r, 'threads': $t, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms']}))" "$line" >> "$OUT"
  done
done
