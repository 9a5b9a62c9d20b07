# round 3c: full GPU suite (W1 fix, chunked host path), W1 A/B, default bench (pcie_inclusive = chunked host path)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/r03c_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python -u tools/exp_gr_tail.py 1000000 717277 >> gpurun_out/r03c_w1_ab.jsonl 2>>gpurun_out/r03c_w1_ab.err || exit 1
  ART_W1=0 timeout -k 10 120 python -u tools/exp_gr_tail.py 1000000 717277 | sed 's/^/W1off /' >> gpurun_out/r03c_w1_ab.jsonl 2>>gpurun_out/r03c_w1_ab.err || exit 1
done
timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --steps 3 --no-cpu-baseline --no-pcie > gpurun_out/r03c_bench_gr.json 2>>gpurun_out/r03c_w1_ab.err || exit 1
ART_W1=0 timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --steps 3 --no-cpu-baseline --no-pcie > gpurun_out/r03c_bench_gr_w1off.json 2>>gpurun_out/r03c_w1_ab.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03c_bench.json 2> gpurun_out/r03c_bench.err || exit 1
echo done
