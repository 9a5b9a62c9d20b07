# round 3o: full GPU suite on the mixed-contraction library; host-path timeline (kernels +
# copies) for the chunked pipeline; scan with the default donation; GR lone-ray tail
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/r03o_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
ART_HOST_TRACE=1 timeout -k 10 300 python -u tools/exp_host_path.py 10000000 1,1 8,3 8,2 > gpurun_out/r03o_host_path.jsonl 2> gpurun_out/r03o_host_path.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r03o_hosttl -o tl -- python3 -u tools/exp_host_path.py 10000000 8,3 > gpurun_out/r03o_hosttl.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/exp_scan_streams.py 1000000 8 32 16 > gpurun_out/r03o_scan_d16.jsonl 2> gpurun_out/r03o_scan.err || exit 1
TAIL_DONATE=4 timeout -k 10 300 python -u tools/exp_gr_tail.py > gpurun_out/r03o_gr_tail.jsonl 2> gpurun_out/r03o_gr_tail.err || exit 1
timeout -k 10 300 python -u tools/exp_sampler_time.py > gpurun_out/r03o_sampler_time.jsonl 2> gpurun_out/r03o_sampler.err || exit 1
echo done
