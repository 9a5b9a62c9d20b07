#!/bin/bash
# Dev: streamed pipeline with free block slots (16, 32) against the CU-masked variant (R = 8)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_edges.py -m gpu -x -q -k streamed --timeout 120 --timeout-method thread > gpurun_out/${1}_pytest.log 2>&1 || exit 1
ART_HOST_STREAM_TIMEOUT_MS=3000 ART_HOST_TRACE=1 timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream stream:0:32 stream:8 single > gpurun_out/${1}.jsonl 2> gpurun_out/${1}.err || exit 1
echo done
