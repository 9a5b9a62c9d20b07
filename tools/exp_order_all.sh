set -o pipefail
for r in 3 4 5 6; do
  for lib in base tools/ab/libart_order.so; do
    if [ "$lib" = base ]; then E=X=1; else E=ART_LIB=$lib; fi
    env $E timeout -k 10 400 python3 -u bench.py --config gr --rays 1000000 --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['device_resident_in_flight']; o=d['device_resident']; print(json.dumps({'lib': '$lib', 'r': $r, 'host_ms': d['ms_per_step'], 'dev_one_ms': o['roofline']['kernel_ms'], 'many_value': m['value'], 'many_ms': m['ms_per_step']}))" >> gpurun_out/order_all.jsonl || exit 1
  done
done
