set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03a_pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u bench.py > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err && \
(ART_LIB=tools/build/libart_w1dbg.so AMD_LOG_LEVEL=3 timeout -k 10 120 python -u tools/exp_axn_case.py flat 1 2000 8 > gpurun_out/r03a_w1dbg.log 2>&1; echo "w1dbg rc=$?")
