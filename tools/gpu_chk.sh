cd "$GRAFT_REPO_ROOT" || exit 1
for lib in "$@"; do
  ART_LIB=$lib timeout -k 10 120 python3 tools/ab_check.py 1000000 2>/dev/null >> gpurun_out/chk.log || exit 1
done
