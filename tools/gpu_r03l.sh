set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tail_donation.py tests/test_edges.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03l_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
ART_LIB=tools/build/libart_trace.so timeout -k 10 200 python -u tools/exp_tail_trace_batch.py flat 8000 > gpurun_out/r03l_trace_flat.jsonl 2>gpurun_out/r03l_trace.err || exit 1
ART_LIB=tools/build/libart_trace.so timeout -k 10 200 python -u tools/exp_tail_trace_batch.py gr 8000 > gpurun_out/r03l_trace_gr.jsonl 2>>gpurun_out/r03l_trace.err || exit 1
echo done
