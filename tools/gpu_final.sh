#!/bin/bash
# Round-end evidence for profiles/: the GPU test suite, smoke, the PMC passes of this library
# build (so bench.py reports roofline.traffic), the default bench line (the host path, with its
# in-kernel span stamps), a rocprofv3 kernel-trace summary of the same command (and one with the
# memory-copy trace: the download copies as blit kernels), the 8-GPU shard size on one GPU,
# configs[3] as one GR batch with its PMC set, and the scan / sampler / tail-ray / host-path /
# small-batch / event / section side figures.
# Usage: TAG=r05fin bash tools/gpu_final.sh [STEP ...]   (no steps: all of them, in order)
# Before a call, on the CPU: build the library (python -c "import __graft_entry__ as g; g.build()") and
# the two section-timing variants the `sections` step loads from the same source (a variant built from
# older source lacks newer symbols and fails to load):
#   python adiabatic_raytracer_amd/build.py --variant tools/ab/libart_sect.so -DART_SECTION_TIMING
#   python adiabatic_raytracer_amd/build.py --variant tools/ab/libart_ssec.so -DART_SAMPLER_SECTIONS
# (.gpurunignore keeps tools/ab/*.so off other pushes: drop that line for a call with `sections`)
# Writes gpurun_out/TAG_*; every GPU step has its own time limit; the first failure ends the run.
TAG=${TAG:-r05fin}
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/${TAG}
run_step() {
  case "$1" in
    pytest)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > ${O}_pytest_gpu.log 2>&1
      rc=$?; [ $rc -le 1 ] ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 ;;
    pmc)
      bash tools/pmc_passes.sh ${O}_pmc 10000000 > ${O}_pmc.log 2>&1 && cp ${O}_pmc/pmc_summary.json profiles/pmc_summary.json ;;
    bench)
      timeout -k 10 600 python3 -u bench.py > ${O}_bench_flat1e7.json 2> ${O}_bench.err ;;
    rocprof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d ${O}_prof -o prof --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > ${O}_bench_prof.json 2> ${O}_prof.err ;;
    rocprof_copies)
      timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d ${O}_profmc -o prof --output-format csv -- python3 bench.py --steps 5 --no-cpu-baseline --no-device > ${O}_bench_profmc.json 2> ${O}_profmc.err ;;
    shard)
      timeout -k 10 300 python3 -u bench.py --rays 1250000 --steps 20 --warmup 5 --no-cpu-baseline > ${O}_bench_1250000.json 2> ${O}_shard.err &&
      timeout -k 10 300 python3 -u bench.py --rays 1250000 --steps 20 --warmup 5 --no-cpu-baseline --no-device --inflight 1 > ${O}_bench_1250000_inflight1.json 2>> ${O}_shard.err ;;
    gr)
      timeout -k 10 600 python3 -u bench.py --config gr --rays 1000000 --steps 5 --no-cpu-baseline > ${O}_bench_gr1e6.json 2> ${O}_gr.err ;;
    pmc_gr)
      bash tools/pmc_gr.sh ${O}_pmc_gr > ${O}_pmc_gr.log 2>&1 ;;
    scan)
      timeout -k 10 300 python3 -u tools/exp_scan_streams.py 1000000 8 32 16 > ${O}_param_scan_1e6_8streams.jsonl 2> ${O}_scan.err ;;
    sampler)
      timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sampler_time.jsonl 2> ${O}_sampler.err ;;
    tail)
      TAIL_DONATE=4 timeout -k 10 300 python3 -u tools/exp_gr_tail.py > ${O}_gr_tail.jsonl 2> ${O}_gr_tail.err ;;
    host)
      ART_HOST_TRACE=1 timeout -k 10 200 python3 -u tools/exp_host_path.py 10000000 stream single > ${O}_host_path.jsonl 2> ${O}_host_path.err ;;
    small)
      timeout -k 10 300 python3 -u tools/exp_small_batch.py > ${O}_small_batch.jsonl 2>> ${O}.err ;;
    events)
      timeout -k 10 300 python3 -u tools/exp_events.py flat 1000,10000,100000 0 > ${O}_events_flat.jsonl 2>> ${O}.err &&
      timeout -k 10 300 python3 -u tools/exp_events.py gr 1000,10000 0 > ${O}_events_gr.jsonl 2>> ${O}.err ;;
    sections)
      ART_LIB=tools/ab/libart_sect.so timeout -k 10 200 python3 -u tools/exp_sections.py > ${O}_sections.jsonl 2>> ${O}.err &&
      ART_LIB=tools/ab/libart_ssec.so timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sampler_sections.jsonl 2> ${O}_sampler_sections.err ;;
    *) echo "unknown step $1"; return 2 ;;
  esac
}
steps=("$@")
[ ${#steps[@]} -gt 0 ] || steps=(pytest smoke pmc bench rocprof shard gr pmc_gr scan sampler tail host small events sections)
for s in "${steps[@]}"; do
  echo "[$(date +%T)] $s"
  run_step "$s" || { echo "[$(date +%T)] $s failed"; exit 1; }
done
echo "[$(date +%T)] done"
