# round 3t: re-entry evidence for the library as committed (162785b): the full GPU suite,
# smoke, the default bench line, its rocprof summary, the sampler, GR and host-path figures
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/r03t_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03t_smoke.log 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03t_bench_flat1e7.json 2> gpurun_out/r03t_bench.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r03t_prof -o prof --output-format csv -- python3 bench.py --steps 5 --no-cpu-baseline --no-pcie > gpurun_out/r03t_bench_prof.json 2>&1 || exit 1
timeout -k 10 300 python -u tools/exp_sampler_time.py > gpurun_out/r03t_sampler_time.jsonl 2> gpurun_out/r03t_sampler.err || exit 1
TAIL_DONATE=4 timeout -k 10 300 python -u tools/exp_gr_tail.py > gpurun_out/r03t_gr_tail.jsonl 2> gpurun_out/r03t_gr_tail.err || exit 1
timeout -k 10 300 python3 -u bench.py --config gr --rays 1000000 --steps 12 --no-cpu-baseline --no-pcie > gpurun_out/r03t_bench_gr1e6.json 2> gpurun_out/r03t_gr.err || exit 1
echo done
