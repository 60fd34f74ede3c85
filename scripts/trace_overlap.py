#!/usr/bin/env python3
"""Batch overlap from a rocprofv3 --kernel-trace csv: per kernel, the average
dispatch duration, the wall span of all its dispatches and the mean number in
flight (sum of durations / union of their intervals).  Consecutive batches run
on their own streams, so a kernel's average duration can exceed the bench's
ms per step: concurrency = avg duration / start-to-start gap.

Usage: trace_overlap.py KERNEL_TRACE_CSV [KERNEL ...]"""
import csv
import json
import sys
from collections import defaultdict

path = sys.argv[1]
want = sys.argv[2:] or ["lean_kernel", "segment_kernel", "plan_query_kernel", "plan_fill_kernel"]
iv = defaultdict(list)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1].strip()
    if name in want:
        iv[name].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
out = {}
for k, v in iv.items():
    v.sort()
    dur = [e - s for s, e in v]
    union, cur_s, cur_e = 0, None, None
    for s, e in v:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        union += cur_e - cur_s
    # the longest run of back-to-back dispatches: the bench's timed loop
    gaps = [v[i + 1][0] - v[i][0] for i in range(len(v) - 1)]
    gaps_sorted = sorted(gaps)
    out[k] = {"dispatches": len(v), "avg_duration_ms": sum(dur) / len(dur) / 1e6,
              "union_ms": union / 1e6, "sum_duration_ms": sum(dur) / 1e6,
              "mean_in_flight": (sum(dur) / union) if union else None,
              "median_start_gap_ms": (gaps_sorted[len(gaps) // 2] / 1e6) if gaps else None}
print(json.dumps(out, indent=1))
