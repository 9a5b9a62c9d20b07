# Evidence set for the library as built: the full GPU suite, smoke, the default bench line, its
# rocprof summary, the sampler, GR and host-path figures. Usage: TAG=r03x bash tools/gpu_evidence.sh
TAG=${TAG:-r03x}
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py > gpurun_out/${TAG}_bench_flat1e7.json 2> gpurun_out/${TAG}_bench.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o prof --output-format csv -- python3 bench.py --steps 5 --no-cpu-baseline --no-pcie > gpurun_out/${TAG}_bench_prof.json 2>&1 || exit 1
timeout -k 10 300 python -u tools/exp_sampler_time.py > gpurun_out/${TAG}_sampler_time.jsonl 2> gpurun_out/${TAG}_sampler.err || exit 1
TAIL_DONATE=4 timeout -k 10 300 python -u tools/exp_gr_tail.py > gpurun_out/${TAG}_gr_tail.jsonl 2> gpurun_out/${TAG}_gr_tail.err || exit 1
timeout -k 10 300 python3 -u bench.py --config gr --rays 1000000 --steps 12 --no-cpu-baseline --no-pcie > gpurun_out/${TAG}_bench_gr1e6.json 2> gpurun_out/${TAG}_gr.err || exit 1
ART_HOST_TRACE=1 timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream single > gpurun_out/${TAG}_host_path.jsonl 2> gpurun_out/${TAG}_host_path.err || exit 1
echo done
