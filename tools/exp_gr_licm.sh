# GR (configs[3]) under the in-tree build and the all-TU no-LICM build: the lone tail ray (717277)
# and the one-batch bench, interleaved (OUT prefix)
for r in 1 2; do
  for lib in base tools/ab/libart_nolicm.so; do
    if [ "$lib" = base ]; then E=X=1; else E=ART_LIB=$lib; fi
    env $E TAIL_DONATE=4 timeout -k 10 200 python3 -u tools/exp_gr_tail.py 1000000 717277 2>/dev/null | tail -1 | sed "s|^|{\"lib\": \"$lib\", \"r\": $r, \"tail\": |; s|$|}|" >> ${OUT}_tail.jsonl || exit 1
    env $E timeout -k 10 300 python3 -u bench.py --config gr --rays 1000000 --steps 3 --warmup 1 --no-cpu-baseline --no-device 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$lib', 'r': $r, 'value': d['value'], 'ms': d['ms_per_step'], 'kms': d['roofline']['kernel_ms']}))" >> ${OUT}_gr.jsonl || exit 1
  done
done
