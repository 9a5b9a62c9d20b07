# round 3f: tail kernel bit-identity A/B (which lane-parallel part differs), sampler change
set -o pipefail
mkdir -p gpurun_out
for lib in default tools/build/libart_tplain.so tools/build/libart_tplaint.so; do
  if [ $lib = default ]; then L=""; else L="ART_LIB=$lib"; fi
  env $L timeout -k 10 300 python -u -m pytest tests/test_gpu_tail_donation.py -m gpu -q -k "is_bit_exact and tail_kernel" --timeout 120 --timeout-method thread > gpurun_out/r03f_tail_$(basename $lib).log 2>&1
  rc=$?; echo "$lib rc=$rc"; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler_prob.py tests/test_gpu_scan_cert.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03f_sampler_tests.log 2>&1
rc=$?; echo "sampler tests rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/exp_sampler_time.py > gpurun_out/r03f_sampler_time.jsonl 2> gpurun_out/r03f_sampler_time.err || exit 1
echo done
timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --streams 1 --donate 16 --steps 3 --no-cpu-baseline --no-pcie > gpurun_out/r03f_bench_gr_s1_d16.json 2>>gpurun_out/r03f_sampler_time.err || exit 1
ART_TAIL=0 timeout -k 10 300 python -u bench.py --config gr --rays 1000000 --streams 1 --donate 16 --steps 3 --no-cpu-baseline --no-pcie > gpurun_out/r03f_bench_gr_s1_d16_notail.json 2>>gpurun_out/r03f_sampler_time.err || exit 1
echo done2
