#!/bin/bash
# Dev: reserved CUs spread over the XCDs or taken from one XCD; streamed and masked single launch
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for x in 0 1; do
  ART_HOST_RESERVE_XCD=$x timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream stream:16 | sed "s|^|xcd$x |" >> gpurun_out/${1}.txt 2>> gpurun_out/${1}.err || exit 1
  ART_HOST_RESERVE_XCD=$x ART_DEV_SINGLE_MASKED=8 timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 single | sed "s|^|xcd$x-masked8 |" >> gpurun_out/${1}.txt 2>> gpurun_out/${1}.err || exit 1
done
timeout -k 10 300 python3 -u -m pytest tests/test_edges.py -m gpu -x -q -k streamed --timeout 120 --timeout-method thread > gpurun_out/${1}_pytest.log 2>&1 || exit 1
echo done
