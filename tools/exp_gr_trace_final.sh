# Kernel trace of configs[3] as one 10^6-ray batch with the final library (hot rays on a side
# stream, the claim order) and the large-batch early-graduation test. OUT prefix.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tail_donation.py -k "large_gr_batch" -m gpu > ${OUT}_test.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d ${OUT}_trace -o kt --output-format csv -- python3 bench.py --config gr --rays 1000000 --steps 1 --warmup 1 --no-cpu-baseline --no-device > ${OUT}_trace.json 2>/dev/null || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}_trace/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "rocclr" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = [i for i, r in enumerate(rows) if "order_keys" in r["Kernel_Name"]][-1]
t0 = int(rows[last]["Start_Timestamp"])
for r in rows[last:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{r['Kernel_Name'][:60]:60s} q{r.get('Queue_Id','?')} start {(s-t0)/1e6:8.2f} end {(e-t0)/1e6:8.2f} ms")
PY
