# the -disable-machine-licm build (in-tree) against the round's previous build: bit identity, then
# interleaved device-kernel and host-path A/B (OUT prefix)
timeout -k 10 300 python3 -u tools/exp_bitident.py ${OUT}_new.npz > ${OUT}_bitident.log 2>&1 &&
BITIDENT_DEVICE_ONLY=1 timeout -k 10 300 python3 -u tools/exp_bitident.py ${OUT}_newdev.npz >> ${OUT}_bitident.log 2>&1 &&
BITIDENT_DEVICE_ONLY=1 ART_LIB=tools/ab/libart_licm_on.so timeout -k 10 300 python3 -u tools/exp_bitident.py ${OUT}_prev.npz >> ${OUT}_bitident.log 2>&1 &&
python3 tools/exp_bitident.py --cmp ${OUT}_newdev.npz ${OUT}_prev.npz >> ${OUT}_bitident.log 2>&1
echo "bitident rc=$?" >> ${OUT}_bitident.log; rm -f ${OUT}_*.npz
ROUNDS=3 bash tools/ab_kernel.sh ${OUT}_ab_device.jsonl base $PREV &&
ROUNDS=3 STEPS=10 bash tools/ab_bench.sh ${OUT}_ab_stream.jsonl base $PREV
