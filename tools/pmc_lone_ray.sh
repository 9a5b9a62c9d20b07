#!/bin/bash
# PMC passes over one lone long ray (the GR batch's ray 717277 alone: one lane of one wave), to
# split its per-attempt time into issued instructions and waiting. One rocprofv3 run per group.
# Usage: tools/pmc_lone_ray.sh OUTDIR [ART_W1=0|1]
OUT=${1:-gpurun_out/pmc_lone}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/pass$i" -o pass$i --output-format csv \
    -- python3 tools/exp_gr_tail.py 1000000 717277 > "$OUT/pass$i.log" 2>&1 || { echo "pass $i ($grp) failed"; exit 1; }
done
echo ok
