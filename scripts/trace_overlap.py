#!/usr/bin/env python3
"""Batch overlap from a rocprofv3 --kernel-trace csv: per kernel, the average
dispatch duration, the wall span of all its dispatches and the mean number in
flight (sum of durations / union of their intervals).  Consecutive batches run
on their own streams, so a kernel's average duration can exceed the bench's
ms per step: concurrency = avg duration / start-to-start gap.

"__device__" (every kernel of the trace): over the middle 60 % of the trace by
dispatch order (the timed loop, away from setup and teardown), the fraction of
the wall time in which at least one kernel runs, and the idle gaps: a GPU that
waits on the host shows up as busy_fraction well under 1.

Usage: trace_overlap.py KERNEL_TRACE_CSV [KERNEL ...]"""
import csv
import json
import sys
from collections import defaultdict

path = sys.argv[1]
want = sys.argv[2:] or ["lean_kernel", "segment_kernel", "plan_query_kernel", "plan_fill_kernel"]
iv = defaultdict(list)
every = []
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1].strip()
    se = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    every.append(se)
    if name in want:
        iv[name].append(se)
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
every.sort()
if len(every) > 10:
    mid = every[len(every) // 5: len(every) * 4 // 5]
    t0, t1 = mid[0][0], max(e for _, e in mid)
    busy, cs, ce, gaps = 0, None, None, []
    for s, e in mid:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
                gaps.append(s - ce)
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    gaps.sort()
    out["__device__"] = {"window_ms": (t1 - t0) / 1e6, "busy_ms": busy / 1e6,
                         "busy_fraction": busy / (t1 - t0) if t1 > t0 else None,
                         "idle_gaps": len(gaps),
                         "idle_gap_p50_us": gaps[len(gaps) // 2] / 1e3 if gaps else 0,
                         "idle_gap_p90_us": gaps[len(gaps) * 9 // 10] / 1e3 if gaps else 0}
print(json.dumps(out, indent=1))
