#!/bin/bash
# Dev: pointwise RHS/condition of two builds compared bit for bit (exp_pointwise_ab.py), then
# integrator A/B (ab_libs.sh) and a host-path settings sweep. Usage: tools/gpu_ab2.sh TAG A.so B.so [more.so]
TAG=$1; A=$2; B=$3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for l in "$A" "$B"; do
  ART_LIB=$l timeout -k 10 120 python3 tools/exp_pointwise_ab.py /tmp/pw_$(basename $l).npz > /dev/null 2>> gpurun_out/${TAG}.err || exit 1
done
python3 tools/cmp_npz.py /tmp/pw_$(basename $A).npz /tmp/pw_$(basename $B).npz > gpurun_out/${TAG}_pointwise.txt 2>&1 || exit 1
shift
REPS=${REPS:-3} NO_GR=${NO_GR:-} timeout -k 10 700 bash tools/ab_libs.sh "$@" > gpurun_out/${TAG}_ab.txt 2>&1 || exit 1
if [ -n "$HOST" ]; then
  timeout -k 10 400 python3 -u tools/exp_host_path.py 10000000 $HOST > gpurun_out/${TAG}_host_path.jsonl 2> gpurun_out/${TAG}_host_path.err || exit 1
fi
echo done
