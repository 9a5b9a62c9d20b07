cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do for s in 8 12 16; do
  timeout -k 10 200 python3 -u bench.py --config gr --rays 1000000 --streams $s --steps 12 --no-cpu-baseline --no-pcie > gpurun_out/r03grv_s${s}_$rep.json 2>> gpurun_out/r03grv.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r03grv_s${s}_$rep.json')); print($s, $rep, d['value'], d['ms_per_step'])"
done; done
