# round 3e: tail kernel correctness (bit-exact donation tests), lone-ray latency, host pipeline v2, GR bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tail_donation.py tests/test_edges.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03e_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  TAIL_DONATE=16 timeout -k 10 120 python -u tools/exp_gr_tail.py 1000000 717277 >> gpurun_out/r03e_tail.jsonl 2>>gpurun_out/r03e_tail.err || exit 1
  timeout -k 10 120 python -u tools/exp_gr_tail.py 1000000 717277 >> gpurun_out/r03e_tail.jsonl 2>>gpurun_out/r03e_tail.err || exit 1
done
ART_HOST_TRACE=1 timeout -k 10 300 python -u tools/exp_host_path.py 10000000 8,3 8,2 4,2 16,3 16,4 > gpurun_out/r03e_host_path.jsonl 2> gpurun_out/r03e_host_path.err || exit 1
timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --steps 3 --no-cpu-baseline --no-pcie > gpurun_out/r03e_bench_gr.json 2>>gpurun_out/r03e_tail.err || exit 1
ART_TAIL=0 timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --steps 3 --no-cpu-baseline --no-pcie > gpurun_out/r03e_bench_gr_notail.json 2>>gpurun_out/r03e_tail.err || exit 1
echo done
