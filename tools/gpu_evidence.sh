#!/bin/bash
# Round-end evidence in one GPU call: tests, smoke, bench and rocprof (tools/gpu_final.sh), the
# PMC passes (tools/pmc_passes.sh) and the side figures (tools/gpu_final2.sh).
# Usage: tools/gpu_evidence.sh TAG
TAG=${1:-r02g}
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_final.sh "$TAG" || exit 1
bash tools/pmc_passes.sh gpurun_out/${TAG}_pmc 10000000 > gpurun_out/${TAG}_pmc.log 2>&1 || exit 1
bash tools/gpu_final2.sh "$TAG" || exit 1
