#!/bin/bash
# Dev: the measured parity margins of the oracle comparisons (ART_PARITY_REPORT), and the GR
# batch with 16 passes in flight
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ART_PARITY_REPORT=$GRAFT_REPO_ROOT/gpurun_out/${1}_parity.jsonl timeout -k 10 600 python3 -u -m pytest tests/test_gpu_propagate.py tests/test_gpu_trees.py tests/test_gpu_saveat.py tests/test_gpu_configs2_full.py tests/test_gpu_tail_donation.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${1}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
echo done
