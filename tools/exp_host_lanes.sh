set -o pipefail
for r in 1 2 3; do
  for v in "base 2" "tools/ab/libart_lanes3.so 2" "tools/ab/libart_lanes3.so 3"; do
    set -- $v
    if [ "$1" = base ]; then E=X=1; else E=ART_LIB=$1; fi
    env $E timeout -k 10 300 python3 -u bench.py --rays 1250000 --steps 20 --warmup 5 --no-cpu-baseline --no-device --inflight $2 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$1', 'inflight': $2, 'r': $r, 'value': d['value'], 'ms': d['ms_per_step']}))" >> gpurun_out/lanes.jsonl || exit 1
  done
done
