#!/bin/bash
# Round-end evidence for profiles/: the GPU test suite, smoke, the PMC passes of this library
# build (so bench.py reports roofline.traffic), the default bench line (the host path, with its
# in-kernel span stamps), a rocprofv3 kernel-trace summary of the same command (and one with the
# memory-copy trace: the download copies as blit kernels), the 8-GPU shard size on one GPU,
# configs[3] as one GR batch with its PMC set, and the scan / sampler / tail-ray / host-path /
# small-batch / event / section side figures.
# Usage: TAG=r05final bash tools/gpu_final.sh   (writes gpurun_out/TAG_*; stops at the first failure)
TAG=${TAG:-r05final}
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
step smoke
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
step pmc
bash tools/pmc_passes.sh gpurun_out/${TAG}_pmc 10000000 > gpurun_out/${TAG}_pmc.log 2>&1 || exit 1
cp gpurun_out/${TAG}_pmc/pmc_summary.json profiles/pmc_summary.json || exit 1
step bench
timeout -k 10 600 python3 -u bench.py > gpurun_out/${TAG}_bench_flat1e7.json 2> gpurun_out/${TAG}_bench.err || exit 1
step rocprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o prof --output-format csv -- python3 bench.py --steps 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_prof.json 2>&1 || exit 1
step rocprof_copies
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/${TAG}_profmc -o prof --output-format csv -- python3 bench.py --steps 5 --no-cpu-baseline --no-device > gpurun_out/${TAG}_bench_profmc.json 2> gpurun_out/${TAG}_profmc.err || exit 1
step shard
timeout -k 10 300 python3 -u bench.py --rays 1250000 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_1250000.json 2> gpurun_out/${TAG}_shard.err || exit 1
timeout -k 10 300 python3 -u bench.py --rays 1250000 --steps 20 --warmup 5 --no-cpu-baseline --no-device --inflight 1 > gpurun_out/${TAG}_bench_1250000_inflight1.json 2>> gpurun_out/${TAG}_shard.err || exit 1
step gr
timeout -k 10 600 python3 -u bench.py --config gr --rays 1000000 --steps 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_gr1e6.json 2> gpurun_out/${TAG}_gr.err || exit 1
step pmc_gr
bash tools/pmc_gr.sh gpurun_out/${TAG}_pmc_gr > gpurun_out/${TAG}_pmc_gr.log 2>&1 || exit 1
step scan
timeout -k 10 300 python3 -u tools/exp_scan_streams.py 1000000 8 32 16 > gpurun_out/${TAG}_param_scan_1e6_8streams.jsonl 2> gpurun_out/${TAG}_scan.err || exit 1
step sampler
timeout -k 10 300 python3 -u tools/exp_sampler_time.py > gpurun_out/${TAG}_sampler_time.jsonl 2> gpurun_out/${TAG}_sampler.err || exit 1
step tail
TAIL_DONATE=4 timeout -k 10 300 python3 -u tools/exp_gr_tail.py > gpurun_out/${TAG}_gr_tail.jsonl 2> gpurun_out/${TAG}_gr_tail.err || exit 1
step host
ART_HOST_TRACE=1 timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream single > gpurun_out/${TAG}_host_path.jsonl 2> gpurun_out/${TAG}_host_path.err || exit 1
step small
timeout -k 10 300 python3 -u tools/exp_small_batch.py > gpurun_out/${TAG}_small_batch.jsonl 2>> gpurun_out/${TAG}.err || exit 1
step events
timeout -k 10 300 python3 -u tools/exp_events.py flat 1000,10000,100000 0 > gpurun_out/${TAG}_events_flat.jsonl 2>> gpurun_out/${TAG}.err || exit 1
timeout -k 10 300 python3 -u tools/exp_events.py gr 1000,10000 0 > gpurun_out/${TAG}_events_gr.jsonl 2>> gpurun_out/${TAG}.err || exit 1
step sections
if [ -f tools/build/libart_sect.so ]; then
  ART_LIB=tools/build/libart_sect.so timeout -k 10 200 python3 -u tools/exp_sections.py > gpurun_out/${TAG}_sections.jsonl 2>> gpurun_out/${TAG}.err || exit 1
fi
step done
echo done
