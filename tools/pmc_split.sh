cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_split
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 -d gpurun_out/pmc_split/p1 -o p1 --output-format csv -- python3 tools/valu_split.py > gpurun_out/pmc_split/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_split/p2 -o p2 --output-format csv -- python3 tools/valu_split.py > gpurun_out/pmc_split/p2.log 2>&1 || exit $?
