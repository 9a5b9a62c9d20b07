#!/bin/bash
# Dev: the donation tests, then an interleaved 1e7-ray flat A/B of the current build against
# the pre-donation build (lone pass, donation off: what the donation code costs unused), then
# bench at 1e6 rays on 3 streams (donation on).
cd "$GRAFT_REPO_ROOT" || exit 1
rm -f gpurun_out/ab_multi.log
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tail_donation.py tests/test_gpu_propagate.py tests/test_gpu_saveat.py > gpurun_out/predon_tests.log 2>&1 || { tail -20 gpurun_out/predon_tests.log; exit 1; }
tail -2 gpurun_out/predon_tests.log
REPS=4 bash tools/ab_multi.sh adiabatic_raytracer_amd/lib/libart.so tools/build/libart_predon.so || exit 1
for r in 1 2; do
timeout -k 10 200 python3 bench.py --rays 1000000 --steps 10 --warmup 2 --no-cpu-baseline --no-pcie 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('1e6', d['value'], d['config'])" || exit 1
done
