#!/bin/bash
# Round-end evidence for profiles/: the GPU test suite, smoke, the default bench line, a
# rocprofv3 kernel-trace summary of the same command, and the GR / 1e6 / scan side figures.
# Usage: tools/gpu_final.sh TAG   (writes gpurun_out/TAG_*; stops at the first failure)
TAG=${1:-r02b}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench_flat1e7.json 2> gpurun_out/${TAG}_bench.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o prof --output-format csv -- python3 bench.py --steps 5 --no-cpu-baseline --no-pcie > gpurun_out/${TAG}_bench_prof.json 2>&1 || exit 1
