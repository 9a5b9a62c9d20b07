# streamed pipeline: integrator blocks left pending behind the helpers' CUs (one line per run)
run() { label=$1; shift
  line=$(env "$@" timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-device --no-cpu-baseline 2>/dev/null | tail -1)
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'label': sys.argv[2], 'value': d['value'], 'ms': d['ms_per_step'], 'kms': d['roofline']['kernel_ms']}))" "$line" "$label" >> $OUT || echo "{\"label\": \"$label\", \"failed\": true}" >> $OUT
}
for r in 1 2; do
  run old_default ART_LIB=tools/ab/libart_r06e.so
  run old_blocks504 ART_LIB=tools/ab/libart_r06e.so ART_HOST_BLOCKS=504
  run old_h16_blocks496 ART_LIB=tools/ab/libart_r06e.so ART_HOST_HELPERS=16 ART_HOST_BLOCKS=496
  run new_h16 X=1
done
