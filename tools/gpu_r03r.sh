# round 3r: host pipeline v4 (finalize writes into mapped pinned memory, preallocated scratch)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_edges.py tests/test_capi.py tests/test_gpu_trees.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03r_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
ART_HOST_TRACE=1 timeout -k 10 300 python -u tools/exp_host_path.py 10000000 1,1 6,2 8,2 10,2 8,3 > gpurun_out/r03r_host_path.jsonl 2> gpurun_out/r03r_host_path.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r03r_hosttl -o tl -- python3 -u tools/exp_host_path.py 10000000 8,2 > gpurun_out/r03r_hosttl.log 2>&1 || exit 1
echo done
