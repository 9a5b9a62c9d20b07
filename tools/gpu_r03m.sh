# round 3m: full suite on the contract=on library, headline bench, donation/tail variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/r03m_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03m_bench.json 2> gpurun_out/r03m_bench.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie --donate 16 > gpurun_out/r03m_bench_d16.json 2>> gpurun_out/r03m_bench.err || exit 1
timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --steps 3 --no-cpu-baseline --no-pcie > gpurun_out/r03m_bench_gr.json 2>> gpurun_out/r03m_bench.err || exit 1
timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --streams 1 --donate 16 --steps 3 --no-cpu-baseline --no-pcie > gpurun_out/r03m_bench_gr_s1.json 2>> gpurun_out/r03m_bench.err || exit 1
timeout -k 10 300 python -u bench.py --rays 1000000 --steps 5 --no-cpu-baseline --no-pcie > gpurun_out/r03m_bench_flat1e6.json 2>> gpurun_out/r03m_bench.err || exit 1
echo done
