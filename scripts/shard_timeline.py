#!/usr/bin/env python3
"""Per kernel name of a rocprofv3 kernel trace: dispatches, mean duration, and
the mean start-to-start gap over the middle 60 % of the trace (the timed loop);
plus the share of wall time with no kernel running.  Usage: TRACE_CSV"""
import csv
import sys
from collections import defaultdict

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0].strip().split("::")[-1][:60]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
n = len(rows)
mid = rows[int(0.2 * n):int(0.8 * n)]
t0, t1 = mid[0][0], max(e for _, e, _ in mid)
by = defaultdict(list)
for s, e, k in mid:
    by[k].append((s, e))
print(f"window {(t1 - t0) / 1e6:.3f} ms, {len(mid)} dispatches")
for k, v in sorted(by.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
    d = sum(e - s for s, e in v) / len(v) / 1e3
    gap = (v[-1][0] - v[0][0]) / max(1, len(v) - 1) / 1e3
    print(f"{k:60s} n {len(v):6d} mean {d:9.1f} us  start gap {gap:8.1f} us")
busy, cs, ce = 0, None, None
for s, e, _ in mid:
    if ce is None or s > ce:
        if ce is not None:
            busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print(f"busy fraction {busy / (t1 - t0):.3f}")
