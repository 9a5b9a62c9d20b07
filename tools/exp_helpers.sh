# streamed pipeline: helper count sweep (one line per run) on the in-tree library and one other
run() { label=$1; shift
  line=$(env "$@" timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-device --no-cpu-baseline 2>/dev/null | tail -1)
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'label': sys.argv[2], 'value': d['value'], 'ms': d['ms_per_step'], 'kms': d['roofline']['kernel_ms'], 'misses': d['config']['host_path_counters']}))" "$line" "$label" >> $OUT || echo "{\"label\": \"$label\", \"failed\": true}" >> $OUT
}
for r in 1 2; do
  run prev ART_LIB=tools/ab/libart_r06e.so
  run h8 ART_HOST_HELPERS=8
  run h16 ART_HOST_HELPERS=16
  run h12 ART_HOST_HELPERS=12
  run h24 ART_HOST_HELPERS=24
done
