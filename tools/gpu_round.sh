#!/bin/bash
# One GPU session: smoke, the GPU test suite, a rocprofv3-profiled bench and the full bench.
# Every GPU step has its own time limit; the chain stops at the first step that crashes,
# faults or times out (ordinary pytest failures, rc 1, do not stop it).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv \
  -- python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
timeout -k 10 240 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
[ -n "$ART_PMC" ] && { bash tools/pmc_passes.sh gpurun_out/pmc 10000000 > gpurun_out/pmc.log 2>&1 || exit $?; }
[ -n "$ART_EXTRA" ] && { timeout -k 10 200 python3 $ART_EXTRA > gpurun_out/extra.log 2>&1 || exit $?; }
exit 0
