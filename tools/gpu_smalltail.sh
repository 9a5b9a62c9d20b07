#!/bin/bash
# Dev: the small-batch tail mode -- tests, then per-call latency of small host batches
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_edges.py tests/test_gpu_tail_donation.py tests/test_gpu_propagate.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${1}_pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/exp_small_batch.py > gpurun_out/${1}_small_batch.jsonl 2> gpurun_out/${1}.err || exit 1
echo done
