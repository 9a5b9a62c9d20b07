# round 3d: host transfer rates, the chunked host path's settings, and the lone-ray PMC passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/build/host_copy_bench > gpurun_out/r03d_host_copy.json 2> gpurun_out/r03d_host_copy.err || exit 1
ART_HOST_TRACE=1 timeout -k 10 300 python -u tools/exp_host_path.py 10000000 1,1 8,3 8,2 16,3 > gpurun_out/r03d_host_path.jsonl 2> gpurun_out/r03d_host_path.err || exit 1
bash tools/pmc_lone_ray.sh gpurun_out/r03d_pmc_lone || exit 1
echo done
