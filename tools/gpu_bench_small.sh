cd "$GRAFT_REPO_ROOT" || exit 1
for st in 1 2 3 4; do
  timeout -k 10 200 python3 bench.py --rays 1000000 --steps 20 --warmup 2 --streams $st --no-cpu-baseline --no-pcie 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print($st, d['value'], d['ms_per_step'])" || exit 1
done
timeout -k 10 200 python3 bench.py --rays 1250000 --steps 20 --warmup 2 --no-cpu-baseline --no-pcie 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('1.25e6 auto', d['value'], d['ms_per_step'], d['config'].get('streams'))"
