#!/bin/bash
# PMC collection for the propagate kernel: one rocprofv3 run per counter group, never
# combined with sys/runtime traces. Runs the byte-count calibration kernel first
# (tools/calib_hbm.hip), then the bench workload for one launch per pass: the streamed host
# pipeline's integrator (bench.py's headline) and the device-resident one.
# Usage: tools/pmc_passes.sh OUTDIR RAYS      (stops at the first failed pass)
OUT=${1:-gpurun_out/pmc}; RAYS=${2:-10000000}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT/calib" "$OUT/kernel"
# FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950 ("exceeds the capabilities of the hardware")
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c -d "$OUT/calib/$c" -o calib \
    --output-format csv -- tools/build/calib_hbm > "$OUT/calib_truth.json" 2> "$OUT/calib_$c.log" || exit $?
done
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_ANY"; do
  i=$((i+1))
  # (counter collection serialises the kernels, so the streamed host pipeline must not hand off
  # between concurrent kernels: ART_HOST_STREAM_SERIAL=1 initialises every tile before the
  # integrator and finalizes after it, with no persistent helpers; the integrator's code and
  # traffic are the streamed instantiation's all the same)
  ART_HOST_STREAM_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/kernel/pass$i" -o pass$i \
    --output-format csv -- python3 bench.py --rays "$RAYS" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pass$i.log" 2>&1 \
    || { echo "pass $i ($grp) failed"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" "flat:$RAYS" "$OUT/pmc_summary.json"
