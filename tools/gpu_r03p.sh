# round 3p: sampler (tight b bound, line windows, LDS-resident line) A/B; host pipeline v3
# (dedicated copy streams); GR passes in flight
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler_prob.py tests/test_gpu_scan_cert.py tests/test_edges.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03p_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
for v in head samp3 main; do
  lib=tools/build/libart_$v.so; [ $v = main ] && lib=adiabatic_raytracer_amd/lib/libart.so
  ART_LIB=$lib timeout -k 10 300 python -u tools/exp_sampler_time.py > gpurun_out/r03p_sampler_$v.jsonl 2>> gpurun_out/r03p.err || exit 1
done
ART_HOST_TRACE=1 timeout -k 10 300 python -u tools/exp_host_path.py 10000000 1,1 8,2 8,3 12,2 16,2 6,2 > gpurun_out/r03p_host_path.jsonl 2> gpurun_out/r03p_host_path.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r03p_hosttl -o tl -- python3 -u tools/exp_host_path.py 10000000 8,2 > gpurun_out/r03p_hosttl.log 2>&1 || exit 1
for s in 3 6; do
  timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --streams $s --steps 12 --no-cpu-baseline --no-pcie > gpurun_out/r03p_bench_gr_s$s.json 2>> gpurun_out/r03p.err || exit 1
done
timeout -k 10 300 python -u tools/exp_scan_streams.py 1000000 8 32 16 > gpurun_out/r03p_scan_d16.jsonl 2>> gpurun_out/r03p.err || exit 1
echo done
