set -o pipefail
mkdir -p gpurun_out
ROUNDS=3 bash tools/ab_kernel.sh gpurun_out/sched_kernel.jsonl base tools/ab/libart_ilp.so tools/ab/libart_mem.so && \
ROUNDS=2 bash tools/ab_bench.sh gpurun_out/sched_bench.jsonl base tools/ab/libart_ilp.so tools/ab/libart_mem.so && \
for r in 1 2; do for lib in base tools/ab/libart_grilp.so; do if [ "$lib" = base ]; then E=X=1; else E=ART_LIB=$lib; fi; env $E timeout -k 10 300 python3 -u bench.py --config gr --rays 1000000 --steps 3 --warmup 1 --no-cpu-baseline --no-device 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$lib', 'r': $r, 'value': d['value'], 'ms': d['ms_per_step'], 'kms': d['roofline']['kernel_ms']}))" >> gpurun_out/sched_gr.jsonl || exit 1; done; done
