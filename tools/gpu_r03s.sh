# round 3s: host pipeline v5 (finalize on its own stream into mapped pinned memory,
# coherent vs non-coherent); sampler 2 vs 3 waves with the ocml-free line setup
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_edges.py tests/test_capi.py tests/test_gpu_sampler_prob.py tests/test_gpu_scan_cert.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03s_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
ART_HOST_TRACE=1 timeout -k 10 300 python -u tools/exp_host_path.py 10000000 1,1 6,2 8,2 8,3 > gpurun_out/r03s_host_path.jsonl 2> gpurun_out/r03s_host_path.err || exit 1
ART_HOST_COHERENT=1 timeout -k 10 300 python -u tools/exp_host_path.py 10000000 1,1 8,2 > gpurun_out/r03s_host_path_coh.jsonl 2> gpurun_out/r03s_host_path_coh.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r03s_hosttl -o tl -- python3 -u tools/exp_host_path.py 10000000 8,2 > gpurun_out/r03s_hosttl.log 2>&1 || exit 1
for w in 2 3; do
  ART_SAMPLER_WPS=$w timeout -k 10 300 python -u tools/exp_sampler_time.py > gpurun_out/r03s_sampler_w$w.jsonl 2>> gpurun_out/r03s.err || exit 1
done
echo done
