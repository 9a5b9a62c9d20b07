cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python3 tools/exp_gr_tail.py > gpurun_out/tail_gr.log 2>&1 &&
ART_LIB=tools/build/libart_sect.so timeout -k 10 100 python3 tools/exp_gr_tail.py 1 717277 >> gpurun_out/tail_gr.log 2>&1 &&
TAIL_KW='{"mass_a": 1e-6, "B0": 2e14, "omega_pul": 12.566370614359172, "theta_m": 0.2, "flat": true}' timeout -k 10 200 python3 tools/exp_gr_tail.py > gpurun_out/tail_p6.log 2>&1
