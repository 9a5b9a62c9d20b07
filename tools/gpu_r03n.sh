# round 3n: mixed contraction (RHS fast, the rest per expression): bit-identity, parity, bench, tail policy
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tail_donation.py tests/test_edges.py tests/test_gpu_propagate.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03n_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
ART_LIB=tools/build/libart_trace.so timeout -k 10 200 python -u tools/exp_tail_trace_batch.py flat 8000 > gpurun_out/r03n_trace_flat.jsonl 2>gpurun_out/r03n.err || exit 1
ART_LIB=tools/build/libart_trace.so timeout -k 10 200 python -u tools/exp_tail_trace_batch.py gr 8000 > gpurun_out/r03n_trace_gr.jsonl 2>>gpurun_out/r03n.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie > gpurun_out/r03n_bench.json 2>>gpurun_out/r03n.err || exit 1
for td in 1 4; do
  ART_TAIL_DONATE=$td timeout -k 10 300 python -u bench.py --rays 1000000 --steps 5 --no-cpu-baseline --no-pcie > gpurun_out/r03n_bench_flat1e6_td$td.json 2>>gpurun_out/r03n.err || exit 1
  ART_TAIL_DONATE=$td timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --steps 3 --no-cpu-baseline --no-pcie > gpurun_out/r03n_bench_gr_td$td.json 2>>gpurun_out/r03n.err || exit 1
done
ART_TAIL=0 timeout -k 10 300 python -u bench.py --rays 1000000 --steps 5 --no-cpu-baseline --no-pcie > gpurun_out/r03n_bench_flat1e6_notail.json 2>>gpurun_out/r03n.err || exit 1
ART_TAIL=0 timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --steps 3 --no-cpu-baseline --no-pcie > gpurun_out/r03n_bench_gr_notail.json 2>>gpurun_out/r03n.err || exit 1
timeout -k 10 300 python -u tools/exp_scan_streams.py 1000000 8 32 0 > gpurun_out/r03n_scan_d0.jsonl 2>>gpurun_out/r03n.err || exit 1
ART_TAIL_DONATE=1 timeout -k 10 300 python -u tools/exp_scan_streams.py 1000000 8 32 16 > gpurun_out/r03n_scan_d16.jsonl 2>>gpurun_out/r03n.err || exit 1
echo done
