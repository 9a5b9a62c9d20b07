#!/bin/bash
# Dev: streamed integrator timing builds, every piece in HBM before the launch
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in adiabatic_raytracer_amd/lib/libart.so tools/build/libart_sfl1k.so tools/build/libart_snogate.so tools/build/libart_sboth.so tools/build/libart_swt.so; do
  ART_LIB=$lib ART_HOST_STREAM_SERIAL=1 timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream stream:1 | sed "s|^|$(basename $lib) |" >> gpurun_out/${1}_serial.txt 2>> gpurun_out/${1}.err || exit 1
done
ART_LIB=tools/build/libart_swt.so timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream | sed "s|^|swt-overlapped |" >> gpurun_out/${1}_serial.txt 2>> gpurun_out/${1}.err || exit 1
ART_LIB=tools/build/libart_swt.so timeout -k 10 300 python3 -u -m pytest tests/test_edges.py -m gpu -x -q -k streamed --timeout 120 --timeout-method thread > gpurun_out/${1}_swt_pytest.log 2>&1 || exit 1
echo done
