# Kernel trace of one configs[3] batch (10^6 GR rays, the single host path) with early graduation
# on and off: the bulk, continuation, hot and regular tail launches' start/end (OUT prefix).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for hot in 128 0; do
  ART_HOT_AT=$hot timeout -k 10 300 rocprofv3 --kernel-trace -d ${OUT}_trace_$hot -o kt --output-format csv -- python3 bench.py --config gr --rays 1000000 --steps 1 --warmup 1 --no-cpu-baseline --no-device > ${OUT}_trace_$hot.json 2>/dev/null || exit 1
done
python3 - "$OUT" <<'PY'
import csv, glob, sys
out = sys.argv[1]
for hot in (128, 0):
    f = glob.glob(f"{out}_trace_{hot}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "propagate_kernel" in r["Kernel_Name"] or "tail_kernel" in r["Kernel_Name"] or "helper" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0 = int(rows[-8]["Start_Timestamp"]) if len(rows) > 8 else int(rows[0]["Start_Timestamp"])
    print("hot_at", hot)
    for r in rows[-8:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"  {r['Kernel_Name'][:60]:60s} q{r.get('Queue_Id','?')} grid {r.get('Grid_Size','?')} start {(s-t0)/1e6:8.2f} end {(e-t0)/1e6:8.2f} ms")
PY
