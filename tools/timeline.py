"""Dev: a text timeline of one rocprofv3 --kernel-trace --memory-copy-trace run (csv output):
every kernel and copy of the last `n` events, with start, end and duration in ms relative to
the first of them, its queue/stream and name -- to see where a pipeline idles.
Usage: timeline.py DIR [n]   (DIR holds *_kernel_trace.csv and *_memory_copy_trace.csv)"""
import csv
import glob
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 80
ev = []
for f in glob.glob(os.path.join(d, "*_kernel_trace.csv")):
    for k in csv.DictReader(open(f)):
        ev.append((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), "K", f"q{k['Queue_Id']} s{k['Stream_Id']}",
                   k["Kernel_Name"][:48]))
for f in glob.glob(os.path.join(d, "*_memory_copy_trace.csv")):
    for m in csv.DictReader(open(f)):
        ev.append((int(m["Start_Timestamp"]), int(m["End_Timestamp"]), "M", f"s{m['Stream_Id']}",
                   m["Direction"].replace("MEMORY_COPY_", "")))
ev.sort()
ev = ev[-n:]
t0 = ev[0][0]
print(f"{'start':>8} {'end':>8} {'ms':>7}  kind queue/stream name")
for a, b, kind, q, name in ev:
    print(f"{(a - t0) / 1e6:8.2f} {(b - t0) / 1e6:8.2f} {(b - a) / 1e6:7.2f}  {kind} {q:8s} {name}")
