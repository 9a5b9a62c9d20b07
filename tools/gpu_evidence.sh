cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_final.sh r02g || exit 1
bash tools/pmc_passes.sh gpurun_out/r02g_pmc 10000000 > gpurun_out/r02g_pmc.log 2>&1 || exit 1
bash tools/gpu_final2.sh r02g || exit 1
