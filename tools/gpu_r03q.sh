# round 3q: host pipeline v3b (uploads submitted before downloads); passes in flight for the
# 1e7 headline, the 1.25e6 shard and the GR batch
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ART_HOST_TRACE=1 timeout -k 10 300 python -u tools/exp_host_path.py 10000000 1,1 8,2 8,3 6,2 12,2 > gpurun_out/r03q_host_path.jsonl 2> gpurun_out/r03q_host_path.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r03q_hosttl -o tl -- python3 -u tools/exp_host_path.py 10000000 8,2 > gpurun_out/r03q_hosttl.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie > gpurun_out/r03q_bench_s1.json 2>> gpurun_out/r03q.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie --streams 2 --steps 6 > gpurun_out/r03q_bench_s2.json 2>> gpurun_out/r03q.err || exit 1
for s in 3 4 6; do
  timeout -k 10 300 python -u bench.py --rays 1250000 --streams $s --steps 12 --no-cpu-baseline --no-pcie > gpurun_out/r03q_bench_1p25e6_s$s.json 2>> gpurun_out/r03q.err || exit 1
done
for s in 4 8; do
  timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --streams $s --steps 16 --no-cpu-baseline --no-pcie > gpurun_out/r03q_bench_gr_s$s.json 2>> gpurun_out/r03q.err || exit 1
done
echo done
