#!/usr/bin/env python3
"""A stretch of the kernel timeline from a rocprofv3 --kernel-trace csv: the
dispatches around the middle of the trace (the timed loop of a long bench
run), one line each -- kernel, queue / stream, start and end relative to the
first shown, duration, grid -- and per kernel the mean duration there.

Usage: timeline.py KERNEL_TRACE_CSV [N_SHOWN=60]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
mid = len(rows) // 2
sel = rows[mid:mid + n]
t0 = int(sel[0]["Start_Timestamp"])
print("cols:", ",".join(k for k in rows[0].keys())[:400])
for r in sel:
    name = r["Kernel_Name"].split("(")[0].replace("wiser::", "").replace("void ", "")[:34]
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{name:34s} q={r.get('Queue_Id','?'):>3s} st={r.get('Stream_Id','?'):>3s} "
          f"start={s/1e3:9.1f}us end={e/1e3:9.1f}us dur={(e-s)/1e3:7.1f}us grid={r.get('Grid_Size_X', r.get('Grid_Size','?'))}")
span = int(sel[-1]["End_Timestamp"]) - t0
per = defaultdict(list)
for r in sel:
    per[r["Kernel_Name"].split("(")[0][-30:]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
print(f"span {span/1e3:.1f}us for {n} dispatches")
for k, v in per.items():
    print(f"  {k:30s} n={len(v)} mean={sum(v)/len(v)/1e3:.1f}us")
