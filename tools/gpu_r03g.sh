# round 3g: tail kernel bit-identity after matching the bulk kernel's glue roundings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tail_donation.py tests/test_edges.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03g_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
ART_LIB=tools/build/libart_tplain.so timeout -k 10 300 python -u -m pytest tests/test_gpu_tail_donation.py -m gpu -q -k "is_bit_exact and tail_kernel" --timeout 120 --timeout-method thread > gpurun_out/r03g_tplain.log 2>&1
rc=$?; echo "tplain rc=$rc"; [ $rc -le 1 ] || exit $rc
TAIL_DONATE=16 timeout -k 10 120 python -u tools/exp_gr_tail.py 1000000 717277 >> gpurun_out/r03g_tail.jsonl 2>>gpurun_out/r03g_tail.err || exit 1
timeout -k 10 120 python -u tools/exp_gr_tail.py 1000000 717277 >> gpurun_out/r03g_tail.jsonl 2>>gpurun_out/r03g_tail.err || exit 1
echo done
