python3 - <<'PY'
import os, glob
print("affinity", len(os.sched_getaffinity(0)), sorted(os.sched_getaffinity(0))[:8], "...")
for p in glob.glob('/sys/class/drm/card*/device/numa_node'):
    try: print(p, open(p).read().strip())
    except Exception as e: print(p, e)
for p in sorted(glob.glob('/sys/devices/system/node/node*/cpulist')):
    print(p, open(p).read().strip())
print("nproc", os.cpu_count())
PY
