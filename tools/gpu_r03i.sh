set -o pipefail
mkdir -p gpurun_out
ART_LIB=tools/build/libart_trace.so timeout -k 10 120 python -u tools/exp_tail_trace.py gr 717277 > gpurun_out/r03i_trace_gr.jsonl 2>gpurun_out/r03i_trace.err || exit 1
ART_LIB=tools/build/libart_trace.so timeout -k 10 120 python -u tools/exp_tail_trace.py flat 758009 > gpurun_out/r03i_trace_flat.jsonl 2>>gpurun_out/r03i_trace.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_tail_donation.py tests/test_edges.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03i_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
TAIL_DONATE=16 timeout -k 10 120 python -u tools/exp_gr_tail.py 1000000 717277 >> gpurun_out/r03i_tail.jsonl 2>>gpurun_out/r03i_trace.err || exit 1
timeout -k 10 120 python -u tools/exp_gr_tail.py 1000000 717277 >> gpurun_out/r03i_tail.jsonl 2>>gpurun_out/r03i_trace.err || exit 1
echo done
