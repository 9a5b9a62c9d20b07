# The hot rule's first test: ART_HOT_AT 128 (default) against 64 (with the default ART_HOT_DTAU and
# with 15.5, which flags fewer rays at 64 attempts), configs[3] as one batch, interleaved (OUT file).
set -o pipefail
for r in 1 2 3; do
  for v in "128 15.95" "64 15.95" "64 15.5"; do
    set -- $v
    ART_HOT_AT=$1 ART_HOT_DTAU=$2 timeout -k 10 300 python3 -u bench.py --config gr --rays 1000000 --steps 3 --warmup 1 --no-cpu-baseline --no-device 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'hot_at': $1, 'dtau': $2, 'r': $r, 'value': d['value'], 'ms': d['ms_per_step'], 'kms': d['roofline']['kernel_ms']}))" >> "$OUT" || exit 1
  done
done
