run() { # label env...
  label=$1; shift
  line=$(env "$@" timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-device --no-cpu-baseline 2>/dev/null | tail -1) || return 1
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'label': sys.argv[2], 'value': d['value'], 'ms': d['ms_per_step'], 'kms': d['roofline']['kernel_ms']}))" "$line" "$label" >> gpurun_out/r06e_matrix.jsonl
}
for r in 1 2; do
run default X=1 || exit 1
run init_all ART_HOST_INIT_RAYS=10000000 || exit 1
run helpers4 ART_HOST_HELPERS=4 || exit 1
run helpers12 ART_HOST_HELPERS=12 || exit 1
run serial ART_HOST_STREAM_SERIAL=1 || exit 1
done
