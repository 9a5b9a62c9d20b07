# round 3b: the full GPU suite on the W1-fixed library, then the 1-wave/SIMD A/B (default vs ART_W1=0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03b_pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; exit 1; }
for i in 1 2; do
  timeout -k 10 120 python -u tools/exp_gr_tail.py 1000000 717277 >> gpurun_out/r03b_w1_ab.jsonl 2>>gpurun_out/r03b_w1_ab.err || exit 1
  ART_W1=0 timeout -k 10 120 python -u tools/exp_gr_tail.py 1000000 717277 | sed 's/^/W1off /' >> gpurun_out/r03b_w1_ab.jsonl 2>>gpurun_out/r03b_w1_ab.err || exit 1
done
timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --steps 3 --no-cpu-baseline --no-pcie > gpurun_out/r03b_bench_gr.json 2>>gpurun_out/r03b_w1_ab.err || exit 1
ART_W1=0 timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --steps 3 --no-cpu-baseline --no-pcie > gpurun_out/r03b_bench_gr_w1off.json 2>>gpurun_out/r03b_w1_ab.err || exit 1
echo done
