#!/bin/bash
# Dev: where the streamed integrator loses time: uploads overlapped or not, reserved CUs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream stream:1 single > gpurun_out/${1}_host_path.jsonl 2> gpurun_out/${1}_host_path.err || exit 1
ART_HOST_STREAM_SERIAL=1 timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream stream:1 > gpurun_out/${1}_host_path_serial.jsonl 2> gpurun_out/${1}_host_path_serial.err || exit 1
echo done
