#!/bin/bash
# Dev: first GPU runs of the streamed host pipeline (tests, then the 1e7-ray timings) and the
# sampler's parity tests for the current build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_edges.py -m gpu -x -v -k "streamed or chunked" --timeout 120 --timeout-method thread > gpurun_out/${1}_pytest_stream.log 2>&1 || exit 1
ART_HOST_TRACE=1 timeout -k 10 300 python3 -u tools/exp_host_path.py 10000000 stream stream:16 single > gpurun_out/${1}_host_path.jsonl 2> gpurun_out/${1}_host_path.err || exit 1


echo done
