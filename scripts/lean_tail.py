#!/usr/bin/env python3
"""Where a headline batch's lean kernel spends its tail (diagnostic; needs a
build whose lean waves write their start and end times into stats words 2
and 3 -- scripts/gpu_lean_tail.sh makes one with scripts/build_variant.py).

Runs C3 headline batches one at a time and pipelined, reads every lean
wave's [start, end] (s_memrealtime, 100 MHz) from wsr_debug_wg_stats and
prints, per batch, the kernel span, the wave-end percentiles relative to the
first wave's start, and how much of the span only a few waves are still
running.  Prints one JSON line."""
import ctypes as C
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import bench  # noqa: E402
import wiser_amd as w  # noqa: E402
from wiser_amd import _capi  # noqa: E402
from wiser_amd._capi import lib  # noqa: E402


def waves(eng, b):
    n_wg, stride = C.c_int32(), C.c_int32()
    lib.wsr_debug_wg_stats(eng._h, b._b, None, 0, C.byref(n_wg), C.byref(stride))
    buf = (C.c_uint32 * (n_wg.value * stride.value))()
    _capi.check(lib.wsr_debug_wg_stats(eng._h, b._b, buf, len(buf), C.byref(n_wg), C.byref(stride)))
    rows = [(buf[i * stride.value + 2], buf[i * stride.value + 3]) for i in range(n_wg.value)]
    # the variant's general workgroups write word 3 = 0; lean waves their times
    return [(s, e) for s, e in rows if e != 0 and e >= s]


def summary(ws):
    t0 = min(s for s, _ in ws)
    ends = sorted(e - t0 for _, e in ws)
    starts = sorted(s - t0 for s, _ in ws)
    span = ends[-1]
    pct = lambda v, q: v[min(len(v) - 1, int(q * len(v)))] / 100.0   # 10 ns ticks -> us
    # time during which fewer than 10 % of the waves are still running
    n = len(ends)
    thin = (ends[-1] - ends[int(0.9 * n)]) / 100.0
    return {"waves": n, "span_us": span / 100.0, "start_p50_us": pct(starts, 0.5), "start_p99_us": pct(starts, 0.99),
            "end_p10_us": pct(ends, 0.1), "end_p50_us": pct(ends, 0.5), "end_p90_us": pct(ends, 0.9),
            "end_p99_us": pct(ends, 0.99), "last_10pct_waves_us": thin}


def main():
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    idx, qlog, _ = bench.ensure_c3(a)
    lines = [l.split() for l in open(qlog).read().splitlines()]
    eng = w.VacuumEngine(idx, device=0, threads=16, positions=False)
    eng.Load()
    bs = []
    for s in range(0, 8 * a.batch, a.batch):
        b = w.ResidentBatch(eng, a.batch, a.k)
        b.upload(bench.resolve(eng, lines[s:s + a.batch], a.k))
        bs.append(b)
    out = {"alone": [], "pipelined": []}
    for b in bs:   # one at a time
        b.run()
        b.fetch()
        out["alone"].append(summary(waves(eng, b)))
    for _ in range(3):   # back to back, as the timed loop runs them
        for b in bs:
            b.run()
    w.sync(eng)
    for b in bs:
        out["pipelined"].append(summary(waves(eng, b)))
    print(json.dumps(out))
    for b in bs:
        b.close()
    eng.close()


if __name__ == "__main__":
    main()
