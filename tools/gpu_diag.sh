cd "$GRAFT_REPO_ROOT" || exit 1
for lib in tools/build/libart_base.so adiabatic_raytracer_amd/lib/libart.so; do
  ART_LIB=$lib timeout -k 10 300 python3 tools/exp_scanpt_diag.py 384 >> gpurun_out/diag.log 2>&1 || exit 1
done
