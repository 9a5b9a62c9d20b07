# bit identity of the in-tree build against $PREV on the device path (flat, GR, oblique GR), then
# the GR one-batch bench and the flat host-path bench, interleaved (OUT prefix)
BITIDENT_DEVICE_ONLY=1 timeout -k 10 300 python3 -u tools/exp_bitident.py ${OUT}_a.npz > ${OUT}_bitident.log 2>&1 &&
BITIDENT_DEVICE_ONLY=1 ART_LIB=$PREV timeout -k 10 300 python3 -u tools/exp_bitident.py ${OUT}_b.npz >> ${OUT}_bitident.log 2>&1 &&
python3 tools/exp_bitident.py --cmp ${OUT}_a.npz ${OUT}_b.npz >> ${OUT}_bitident.log 2>&1
echo "bitident rc=$?" >> ${OUT}_bitident.log; rm -f ${OUT}_*.npz
for r in 1 2; do
  for lib in base $PREV; do
    if [ "$lib" = base ]; then E=X=1; else E=ART_LIB=$lib; fi
    env $E timeout -k 10 300 python3 -u bench.py --config gr --rays 1000000 --steps 3 --warmup 1 --no-cpu-baseline --no-device 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$lib', 'r': $r, 'cfg': 'gr', 'value': d['value'], 'ms': d['ms_per_step'], 'kms': d['roofline']['kernel_ms']}))" >> ${OUT}_ab.jsonl || exit 1
    env $E timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-device 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$lib', 'r': $r, 'cfg': 'flat', 'value': d['value'], 'ms': d['ms_per_step'], 'kms': d['roofline']['kernel_ms']}))" >> ${OUT}_ab.jsonl || exit 1
  done
done
