#!/bin/bash
# PMC set of configs[3]: the bulk, continuation and tail kernels of one 1e6-ray
# GR batch (bench.py --config gr, one host call), and ray 717277 alone on the one-wave-per-ray tail
# kernel (tools/exp_gr_tail.py). One rocprofv3 run per counter group, nothing else traced.
# Usage: tools/pmc_gr.sh OUTDIR      (stops at the first failed pass)
OUT=${1:-gpurun_out/pmc_gr}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/batch/pass$i" -o p --output-format csv -- \
    python3 bench.py --config gr --rays 1000000 --steps 1 --warmup 0 --no-cpu-baseline --no-device \
    > "$OUT/batch_pass$i.log" 2>&1 || { echo "batch pass $i ($grp) failed"; exit 1; }
  TAIL_DONATE=4 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/tail/pass$i" -o p --output-format csv -- \
    python3 tools/exp_gr_tail.py 1000000 717277 > "$OUT/tail_pass$i.log" 2>&1 || { echo "tail pass $i ($grp) failed"; exit 1; }
done
python3 tools/pmc_table.py "$OUT/batch" "propagate_kernel|tail_kernel" "$OUT/gr_batch_pmc.json" > /dev/null &&
python3 tools/pmc_table.py "$OUT/tail" "tail_kernel" "$OUT/gr_tail_pmc.json" > /dev/null
