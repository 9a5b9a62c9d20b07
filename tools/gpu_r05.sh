#!/bin/bash
# Round-5 GPU session steps. Usage: TAG=r05a bash tools/gpu_r05.sh STEP [STEP ...]
# (Dev session log of round 5. Variant libraries named by the steps are built with
# `python adiabatic_raytracer_amd/build.py --variant tools/build/libart_X.so -DSWITCH`; the steps whose
# switch was removed after its A/B are kept as the record of how the r05* profiles were made.)
# Every GPU step runs under its own time limit; the first failure ends the session.
TAG=${TAG:-r05}
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/${TAG}
say() { echo "[$(date +%T)] $*"; }
run_step() {
  case "$1" in
    pytest)  # the whole GPU suite
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > ${O}_pytest_gpu.log 2>&1 ;;
    pytest_rehearsal)
      timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs2_full.py -m gpu -v -k rehearsal --timeout 300 --timeout-method thread > ${O}_pytest_rehearsal.log 2>&1 ;;
    pytest_host)  # the host paths: streamed, give-up, async
      timeout -k 10 600 python3 -u -m pytest tests/test_edges.py tests/test_gpu_async_host.py -m gpu -v --timeout 300 --timeout-method thread > ${O}_pytest_host.log 2>&1 ;;
    pytest_direct)  # the host paths with the pieces' blobs in pinned host memory (ART_HOST_DIRECT=1)
      ART_HOST_DIRECT=1 timeout -k 10 600 python3 -u -m pytest tests/test_edges.py tests/test_gpu_async_host.py -m gpu -v --timeout 300 --timeout-method thread > ${O}_pytest_direct.log 2>&1 ;;
    shard_t1)  # the 8-GPU shard size, one call at a time, traced; then the same with direct blobs
      ART_HOST_TRACE=1 timeout -k 10 300 python3 -u bench.py --rays 1250000 --steps 10 --warmup 2 --no-cpu-baseline --no-device --inflight 1 > ${O}_bench_1250000_if1_trace.json 2> ${O}_shard_if1_trace.err &&
      ART_HOST_DIRECT=1 ART_HOST_TRACE=1 timeout -k 10 300 python3 -u bench.py --rays 1250000 --steps 10 --warmup 2 --no-cpu-baseline --no-device --inflight 1 > ${O}_bench_1250000_if1_direct_trace.json 2> ${O}_shard_if1_direct_trace.err ;;
    ab_direct)  # interleaved: host pipeline with download copies vs direct blobs, 1e7 and 1.25e6, one call in flight
      for r in 1 2; do
        for dm in 0 1; do
          ART_HOST_DIRECT=$dm timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-device --steps 10 --warmup 2 --inflight 1 > ${O}_abd_1e7_d${dm}_r$r.json 2>> ${O}_ab_direct.err || return 1
          ART_HOST_DIRECT=$dm timeout -k 10 300 python3 -u bench.py --rays 1250000 --no-cpu-baseline --no-device --steps 10 --warmup 2 --inflight 1 > ${O}_abd_1250000_d${dm}_r$r.json 2>> ${O}_ab_direct.err || return 1
        done
      done ;;
    ab_gr_pf)  # GR 1e6 batch: slot-row prefetch (this build) vs without, interleaved
      for r in 1 2; do
        timeout -k 10 300 python3 -u bench.py --config gr --rays 1000000 --steps 5 --warmup 1 --no-cpu-baseline --no-device > ${O}_abpf_gr_base_r$r.json 2>> ${O}_ab_gr_pf.err || return 1
        ART_LIB=tools/build/libart_nopf.so timeout -k 10 300 python3 -u bench.py --config gr --rays 1000000 --steps 5 --warmup 1 --no-cpu-baseline --no-device > ${O}_abpf_gr_nopf_r$r.json 2>> ${O}_ab_gr_pf.err || return 1
      done ;;
    fetch_grad)  # device-resident 1e7 launch: FETCH_SIZE with graduation at its default and off
      timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d ${O}_fetch/grad_default -o p --output-format csv -- python3 tools/exp_sections.py > ${O}_fetch_grad_default.log 2>&1 &&
      ART_GRADUATE=0 timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d ${O}_fetch/grad_off -o p --output-format csv -- python3 tools/exp_sections.py > ${O}_fetch_grad_off.log 2>&1 &&
      timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d ${O}_fetch/hit_default -o p --output-format csv -- python3 tools/exp_sections.py > ${O}_fetch_hit_default.log 2>&1 ;;
    shard_fu)  # 1.25e6 rays, one call at a time: first upload unit 2^16 (default) vs 2^18, interleaved; then one traced run
      for r in 1 2; do
        for fu in 65536 262144; do
          ART_HOST_FIRST_UNIT=$fu timeout -k 10 300 python3 -u bench.py --rays 1250000 --no-cpu-baseline --no-device --steps 10 --warmup 2 --inflight 1 > ${O}_fu_${fu}_r$r.json 2>> ${O}_shard_fu.err || return 1
        done
      done &&
      ART_HOST_TRACE=1 timeout -k 10 300 python3 -u bench.py --rays 1250000 --steps 10 --warmup 2 --no-cpu-baseline --no-device --inflight 1 > ${O}_bench_1250000_if1_trace.json 2> ${O}_shard_if1_trace.err ;;
    ab_swps)  # sampler: 2, 3 and 4 waves/SIMD builds, interleaved
      for r in 1 2; do
        for w in 2 3 4; do
          ART_SAMPLER_WPS=$w timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_swps_${w}_r$r.jsonl 2>> ${O}_ab_swps.err || return 1
        done
      done ;;
    ab_host)  # this build vs tools/build/libart_prev.so (the previous commit), interleaved: 1.25e6 with 1 and 2 calls in flight, 1e7
      for r in 1 2; do
        for lib in base prev; do
          if [ $lib = prev ]; then export ART_LIB=tools/build/libart_prev.so; else unset ART_LIB; fi
          timeout -k 10 300 python3 -u bench.py --rays 1250000 --no-cpu-baseline --no-device --steps 10 --warmup 2 --inflight 1 > ${O}_abh_1250000_if1_${lib}_r$r.json 2>> ${O}_ab_host.err &&
          timeout -k 10 300 python3 -u bench.py --rays 1250000 --no-cpu-baseline --no-device --steps 10 --warmup 2 --inflight 2 > ${O}_abh_1250000_if2_${lib}_r$r.json 2>> ${O}_ab_host.err &&
          timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-device --steps 10 --warmup 2 > ${O}_abh_1e7_${lib}_r$r.json 2>> ${O}_ab_host.err || { unset ART_LIB; return 1; }
        done
      done; unset ART_LIB ;;
    shard_trace)  # 1.25e6 rays, one call at a time, traced
      ART_HOST_TRACE=1 timeout -k 10 300 python3 -u bench.py --rays 1250000 --steps 10 --warmup 2 --no-cpu-baseline --no-device --inflight 1 > ${O}_bench_1250000_if1_trace.json 2> ${O}_shard_if1_trace.err ;;
    pytest_sampler)
      timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sampler_prob.py tests/test_gpu_scan_cert.py -m gpu -v --timeout 300 --timeout-method thread > ${O}_pytest_sampler.log 2>&1 ;;
    ab_sampler)  # block-certified sampler (this build, 3 and 2 waves/SIMD) vs the step-by-step one, interleaved
      for r in 1 2; do
        timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sab_block3_r$r.jsonl 2>> ${O}_ab_sampler.err &&
        ART_SAMPLER_WPS=2 timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sab_block2_r$r.jsonl 2>> ${O}_ab_sampler.err &&
        ART_LIB=tools/build/libart_stepwise.so timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sab_step_r$r.jsonl 2>> ${O}_ab_sampler.err || return 1
      done ;;
    sec_sampler)  # sampler section split: blocks of 3, of 2, step by step; and the KB=2 build's time
      for v in ssec ssec_kb2 ssec_step; do
        ART_LIB=tools/build/libart_$v.so timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sec_$v.jsonl 2> ${O}_sec_$v.err || return 1
      done &&
      ART_LIB=tools/build/libart_kb2.so timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sab_kb2.jsonl 2>> ${O}_ab_sampler.err ;;
    scan)  # configs[4]: the 32-point scan, 1e6 rays a point, 8 streams
      timeout -k 10 300 python3 -u tools/exp_scan_streams.py 1000000 8 32 16 > ${O}_param_scan_1e6_8streams.jsonl 2> ${O}_scan.err ;;
    scan_step)  # the same with the step-by-step sampler everywhere
      ART_SAMPLER_BLOCKS=0 timeout -k 10 300 python3 -u tools/exp_scan_streams.py 1000000 8 32 16 > ${O}_param_scan_1e6_8streams_step.jsonl 2> ${O}_scan_step.err ;;
    ab_hprio)  # helper waves at issue priority 2 (dev build) vs this build; and a first init pass of 65536 rays
      for r in 1 2; do
        for lib in base hp; do
          if [ $lib = hp ]; then export ART_LIB=tools/build/libart_hprio.so; else unset ART_LIB; fi
          timeout -k 10 300 python3 -u bench.py --rays 1250000 --no-cpu-baseline --no-device --steps 10 --warmup 2 --inflight 1 > ${O}_ahp_1250000_${lib}_r$r.json 2>> ${O}_ab_hprio.err &&
          ART_HOST_INIT_RAYS=65536 timeout -k 10 300 python3 -u bench.py --rays 1250000 --no-cpu-baseline --no-device --steps 10 --warmup 2 --inflight 1 > ${O}_ahp_1250000_init64k_${lib}_r$r.json 2>> ${O}_ab_hprio.err &&
          timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-device --steps 10 --warmup 2 > ${O}_ahp_1e7_${lib}_r$r.json 2>> ${O}_ab_hprio.err || { unset ART_LIB; return 1; }
        done
      done; unset ART_LIB ;;
    ab_scan)  # the scan: default sampler choice vs blocks of steps for every line, interleaved
      for r in 1 2; do
        timeout -k 10 300 python3 -u tools/exp_scan_streams.py 1000000 8 32 16 > ${O}_scan_default_r$r.jsonl 2>> ${O}_ab_scan.err &&
        ART_SAMPLER_BLOCKS=1 timeout -k 10 300 python3 -u tools/exp_scan_streams.py 1000000 8 32 16 > ${O}_scan_blocks_r$r.jsonl 2>> ${O}_ab_scan.err || return 1
      done ;;
    sweep_init)  # the first init pass's size (ART_HOST_INIT_RAYS; default 2 rays per integrator lane = 258048)
      for r in 1 2; do
        for ir in 32768 65536 131072 258048; do
          ART_HOST_INIT_RAYS=$ir timeout -k 10 300 python3 -u bench.py --rays 1250000 --no-cpu-baseline --no-device --steps 10 --warmup 2 --inflight 1 > ${O}_si_1250000_if1_${ir}_r$r.json 2>> ${O}_sweep_init.err &&
          ART_HOST_INIT_RAYS=$ir timeout -k 10 300 python3 -u bench.py --rays 1250000 --no-cpu-baseline --no-device --steps 10 --warmup 2 --inflight 2 > ${O}_si_1250000_if2_${ir}_r$r.json 2>> ${O}_sweep_init.err &&
          ART_HOST_INIT_RAYS=$ir timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-device --steps 10 --warmup 2 > ${O}_si_1e7_${ir}_r$r.json 2>> ${O}_sweep_init.err || return 1
        done
      done ;;
    fetch_n)  # device-resident launch: FETCH_SIZE per ray at 1e6, 2.5e6 and 1e7 rays (do the init records' re-reads hit the 256 MiB Infinity Cache?)
      for n in 1000000 2500000 10000000; do
        timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d ${O}_fetchn/n$n -o p --output-format csv -- python3 tools/exp_sections.py $n > ${O}_fetchn_$n.log 2>&1 || return 1
      done ;;
    ab_if_1e7)  # the 1e7 headline: one call at a time vs two in flight, interleaved
      for r in 1 2; do
        for f in 1 2; do
          timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-device --steps 10 --warmup 2 --inflight $f > ${O}_if_1e7_${f}_r$r.json 2>> ${O}_ab_if.err || return 1
        done
      done ;;
    ab_sblocks)  # sampler: the default choice (step by step below maxR 60 km) vs blocks for every line, interleaved; and the section split of blocks
      for r in 1 2; do
        timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sb_default_r$r.jsonl 2>> ${O}_ab_sblocks.err &&
        ART_SAMPLER_BLOCKS=1 timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sb_blocks_r$r.jsonl 2>> ${O}_ab_sblocks.err || return 1
      done &&
      ART_SAMPLER_BLOCKS=1 ART_LIB=tools/build/libart_ssec.so timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sec_blocks.jsonl 2> ${O}_sec_blocks.err ;;
    ab_sfin)  # sampler: this build vs the round-5 final library (tools/build/libart_fin.so), interleaved; and blocks forced for every line
      for r in 1 2; do
        timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sf_new_r$r.jsonl 2>> ${O}_ab_sfin.err &&
        ART_LIB=tools/build/libart_fin.so timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sf_fin_r$r.jsonl 2>> ${O}_ab_sfin.err &&
        ART_SAMPLER_BLOCKS=1 timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sf_newblocks_r$r.jsonl 2>> ${O}_ab_sfin.err || return 1
      done ;;
    ab_sill)  # sampler: this build vs the 3-site Illinois variant vs the round-5 final library, interleaved
      for r in 1 2; do
        for lib in base ill3 fin; do
          if [ $lib = base ]; then unset ART_LIB; else export ART_LIB=tools/build/libart_$lib.so; fi
          timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_si_${lib}_r$r.jsonl 2>> ${O}_ab_sill.err || { unset ART_LIB; return 1; }
        done
      done; unset ART_LIB ;;
    ab_numa)  # bench bound to the GPU's NUMA node (default) vs unbound (ART_BENCH_NO_NUMA=1), interleaved
      for r in 1 2 3; do
        for b in bound unbound; do
          if [ $b = unbound ]; then export ART_BENCH_NO_NUMA=1; else unset ART_BENCH_NO_NUMA; fi
          timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-device --steps 10 --warmup 2 > ${O}_an_1e7_${b}_r$r.json 2>> ${O}_ab_numa.err &&
          timeout -k 10 300 python3 -u bench.py --rays 1250000 --no-cpu-baseline --no-device --steps 10 --warmup 2 > ${O}_an_1250000_${b}_r$r.json 2>> ${O}_ab_numa.err || { unset ART_BENCH_NO_NUMA; return 1; }
        done
      done; unset ART_BENCH_NO_NUMA ;;
    ab_helpers)  # helper blocks beside the streamed integrator: 6 / 8 (default) / 12, interleaved
      for r in 1 2 3; do
        for h in 6 8 12; do
          ART_HOST_HELPERS=$h timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-device --steps 10 --warmup 2 > ${O}_ah_1e7_${h}_r$r.json 2>> ${O}_ab_helpers.err &&
          ART_HOST_HELPERS=$h timeout -k 10 300 python3 -u bench.py --rays 1250000 --no-cpu-baseline --no-device --steps 10 --warmup 2 > ${O}_ah_1250000_${h}_r$r.json 2>> ${O}_ab_helpers.err || return 1
        done
      done ;;
    ab_gate)  # calls in flight: the next call's launch gated on the previous integrator being resident (this build) vs not (libart_nogate.so), interleaved
      for r in 1 2 3; do
        for lib in base nogate; do
          if [ $lib = base ]; then unset ART_LIB; else export ART_LIB=tools/build/libart_$lib.so; fi
          timeout -k 10 300 python3 -u bench.py --rays 1250000 --no-cpu-baseline --no-device --steps 20 --warmup 3 > ${O}_ag_1250000_${lib}_r$r.json 2>> ${O}_ab_gate.err || { unset ART_LIB; return 1; }
        done
      done; unset ART_LIB &&
      timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-device --steps 10 --warmup 2 > ${O}_ag_1e7_base.json 2>> ${O}_ab_gate.err ;;
    pytest_edges)
      timeout -k 10 400 python3 -u -m pytest tests/test_edges.py -m gpu -v --timeout 300 --timeout-method thread > ${O}_pytest_edges.log 2>&1 ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 ;;
    bench)  # the default bench line (host path, 1e7 flat)
      timeout -k 10 600 python3 -u bench.py > ${O}_bench_flat1e7.json 2> ${O}_bench.err ;;
    bench_nocpu)
      timeout -k 10 600 python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 2 > ${O}_bench_flat1e7_nocpu.json 2> ${O}_bench_nocpu.err ;;
    rocprof)  # kernel trace of the bench command (no counters)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d ${O}_prof -o prof --output-format csv -- python3 bench.py --steps 5 --no-cpu-baseline > ${O}_bench_prof.json 2> ${O}_prof.err ;;
    rocprof_copies)  # the same with the memory-copy trace: are the pipeline's copies DMA or blit kernels?
      timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d ${O}_profmc -o prof --output-format csv -- python3 bench.py --steps 5 --no-cpu-baseline --no-device > ${O}_bench_profmc.json 2> ${O}_profmc.err ;;
    shard)  # the 8-GPU shard size on one GPU, with the host pipeline's trace
      ART_HOST_TRACE=1 timeout -k 10 300 python3 -u bench.py --rays 1250000 --steps 10 --warmup 2 --no-cpu-baseline > ${O}_bench_1250000.json 2> ${O}_shard_trace.err ;;
    shard1)  # the same, one host call at a time
      timeout -k 10 300 python3 -u bench.py --rays 1250000 --steps 10 --warmup 2 --no-cpu-baseline --inflight 1 > ${O}_bench_1250000_if1.json 2> ${O}_shard1.err ;;
    bench_if2)  # the 1e7 headline workload with two host calls in flight
      timeout -k 10 600 python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --inflight 2 --no-device > ${O}_bench_flat1e7_if2.json 2> ${O}_bench_if2.err ;;
    ab_tail)  # tail kernel: wave-uniform branches (this build) against none and against RHS-uniform too
      ROUNDS=3 bash tools/ab_tail.sh ${O}_ab_tail.jsonl base tools/build/libart_tnouni.so tools/build/libart_trhs.so ;;
    pytest_tail)
      timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tail_donation.py tests/test_longest_ray.py -m gpu -v --timeout 300 --timeout-method thread > ${O}_pytest_tail.log 2>&1 ;;
    ab_pf)  # the slot-row prefetch variant against this build, interleaved
      ROUNDS=3 bash tools/ab_kernel.sh ${O}_ab_prefetch.jsonl base tools/build/libart_pf.so ;;
    ssec)  # the sampler's section split (dev build), flat 1e7 and the scan's largest-maxR point
      ART_LIB=tools/build/libart_ssec.so timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sampler_sections.jsonl 2> ${O}_sampler_sections.err ;;
    sampler)
      timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_sampler_time.jsonl 2> ${O}_sampler.err ;;
    gr)
      timeout -k 10 600 python3 -u bench.py --config gr --rays 1000000 --steps 5 --no-cpu-baseline > ${O}_bench_gr1e6.json 2> ${O}_gr.err ;;
    tail)  # ray 717277 alone on the tail kernel
      TAIL_DONATE=4 timeout -k 10 300 python3 -u tools/exp_gr_tail.py 1000000 717277 > ${O}_gr_tail.jsonl 2> ${O}_gr_tail.err ;;
    grsmall)  # GR batches between 1024 and ncu x 256 rays, donation 16 vs 0
      timeout -k 10 300 python3 -u tools/exp_gr_donate_small.py 4096,16384,65536 > ${O}_gr_donate_small.jsonl 2> ${O}_grsmall.err ;;
    w1)  # occupancy sensitivity: the 1-wave/SIMD integrator on the 1e7 device-resident batch
      ART_LIB=tools/build/libart_w1.so timeout -k 10 300 python3 -u tools/exp_sections.py > ${O}_w1_device.jsonl 2> ${O}_w1.err &&
      timeout -k 10 300 python3 -u tools/exp_sections.py > ${O}_w2_device.jsonl 2>> ${O}_w1.err ;;
    tcc)  # L2 hit/miss of both integrator builds (the fetch question), and FETCH_SIZE twice
      for i in 1 2; do
        ART_HOST_STREAM_SERIAL=1 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d ${O}_tcc/hit$i -o p \
          --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > ${O}_tcc_hit$i.log 2>&1 || return 1
        ART_HOST_STREAM_SERIAL=1 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d ${O}_tcc/fetch$i -o p \
          --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > ${O}_tcc_fetch$i.log 2>&1 || return 1
      done ;;
    pmc_gr)  # configs[3]: bulk, continuation and tail kernels of one batch, and ray 717277 alone
      bash tools/pmc_gr.sh ${O}_pmc_gr > ${O}_pmc_gr.log 2>&1 ;;
    ab_fastsign)  # sampler grid signs from sampler_sign_fast + inner steps (this build, 3 and 2 waves/SIMD) vs tools/build/libart_base.so, interleaved
      for r in 1 2; do
        ART_LIB=tools/build/libart_base.so timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_fs_base_r$r.jsonl 2>> ${O}_ab_fastsign.err &&
        timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_fs_new3_r$r.jsonl 2>> ${O}_ab_fastsign.err &&
        ART_SAMPLER_WPS=2 timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_fs_new2_r$r.jsonl 2>> ${O}_ab_fastsign.err || return 1
      done ;;
    ab_sgrid)  # the 32-point scan with the sampler's grid at 1/d of the block slots (ART_SAMPLER_GRID_DIV), interleaved
      for r in 1 2; do
        for d in 1 2 4 8; do
          ART_SAMPLER_GRID_DIV=$d timeout -k 10 300 python3 -u tools/exp_scan_streams.py 1000000 8 32 16 > ${O}_sgrid_${d}_r$r.jsonl 2>> ${O}_ab_sgrid.err || return 1
        done
      done ;;
    ab_brclass)  # brackets classified when found (this build) vs tools/build/libart_prev.so (fast signs only), interleaved
      for r in 1 2; do
        ART_LIB=tools/build/libart_prev.so timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_bc_prev_r$r.jsonl 2>> ${O}_ab_brclass.err &&
        timeout -k 10 300 python3 -u tools/exp_sampler_time.py > ${O}_bc_new_r$r.jsonl 2>> ${O}_ab_brclass.err &&
        ART_LIB=tools/build/libart_prev.so timeout -k 10 300 python3 -u tools/exp_scan_streams.py 1000000 8 32 16 > ${O}_bc_scan_prev_r$r.jsonl 2>> ${O}_ab_brclass.err &&
        timeout -k 10 300 python3 -u tools/exp_scan_streams.py 1000000 8 32 16 > ${O}_bc_scan_new_r$r.jsonl 2>> ${O}_ab_brclass.err || return 1
      done ;;
    scan_base)  # the 32-point scan with tools/build/libart_base.so
      ART_LIB=tools/build/libart_base.so timeout -k 10 300 python3 -u tools/exp_scan_streams.py 1000000 8 32 16 > ${O}_scan_base.jsonl 2> ${O}_scan_base.err ;;
    pmc)  # the full PMC set of this build (bench.py's roofline.traffic)
      bash tools/pmc_passes.sh ${O}_pmc 10000000 > ${O}_pmc.log 2>&1 ;;
    *) echo "unknown step $1"; return 2 ;;
  esac
}
for s in "$@"; do
  say "$s"
  run_step "$s"
  rc=$?
  say "$s rc=$rc"
  if [ "${s#pytest}" != "$s" ]; then [ $rc -le 1 ] || exit $rc; else [ $rc -eq 0 ] || exit $rc; fi
done
say done
