#!/usr/bin/env python3
"""Where a C3 headline batch's lean waves spend their time (diagnostic; needs
the `leanphase` build of scripts/gpu_lean_phase.sh, whose lean waves write,
per wave, the ticks spent in item segments (stats word 0), in item ends --
re-filter, count hand-off and the query replay of the last item (word 2) --
and the longest single item end (word 3); s_memrealtime, 100 MHz).

Runs 8 headline batches one at a time and then back to back (3 passes), and
prints one JSON line: per batch, the waves' summed segment and end times, the
end share, and the longest item ends."""
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


def rows(eng, b, n_lean_rows):
    n_wg, stride = C.c_int32(), C.c_int32()
    lib.wsr_debug_wg_stats(eng._h, b._b, None, 0, C.byref(n_wg), C.byref(stride))
    buf = (C.c_uint32 * (n_wg.value * stride.value))()
    _capi.check(lib.wsr_debug_wg_stats(eng._h, b._b, buf, len(buf), C.byref(n_wg), C.byref(stride)))
    s = stride.value
    first = max(0, n_wg.value - n_lean_rows)   # (general workgroups first, then lean waves)
    return [tuple(buf[i * s + j] for j in range(4)) for i in range(first, n_wg.value)]


def summary_end(rs):
    """the `endphase` build: word 0 = ticks in item-end re-filters and stores,
    1 = in the count hand-off (store wait + q_done atomic), 2 = in query
    replays, 3 = the longest replay"""
    w = [sum(r[j] for r in rs) / 100.0 for j in range(3)]
    mx = sorted(r[3] / 100.0 for r in rs)
    pct = lambda v, q: v[min(len(v) - 1, int(q * len(v)))]
    return {"waves": len(rs), "refilter_us_sum": round(w[0], 1), "handoff_us_sum": round(w[1], 1),
            "replay_us_sum": round(w[2], 1), "replay_max_us": round(mx[-1], 2),
            "replay_max_p99_us": round(pct(mx, 0.99), 2)}


def summary_count(rs):
    """the `endcount` build: per wave its longest replay's events (word 0) and
    heap insertions (word 1), summed replay ticks (2), longest replay (3)"""
    top = sorted(rs, key=lambda r: -r[3])[:8]
    return {"waves": len(rs), "replay_us_sum": round(sum(r[2] for r in rs) / 100.0, 1),
            "longest": [{"us": r[3] / 100.0, "events": r[0], "inserts": r[1]} for r in top]}


def summary(rs):
    if MODE == "end":
        return summary_end(rs)
    if MODE == "count":
        return summary_count(rs)
    seg = sum(r[0] for r in rs) / 100.0
    fin = sum(r[2] for r in rs) / 100.0
    fmax = sorted(r[3] / 100.0 for r in rs)
    pct = lambda v, q: v[min(len(v) - 1, int(q * len(v)))]
    return {"waves": len(rs), "seg_us_sum": round(seg, 1), "end_us_sum": round(fin, 1),
            "end_share": round(fin / max(1e-9, seg + fin), 4), "end_max_us": round(fmax[-1], 2),
            "end_max_p99_us": round(pct(fmax, 0.99), 2), "end_max_p50_us": round(pct(fmax, 0.5), 2),
            "dblk": sum(r[1] for r in rs)}


MODE = "phase"


def main():
    global MODE
    if sys.argv[1:] in (["--end"], ["--count"]):
        MODE = sys.argv[1][2:]
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    idx, qlog, _ = bench.ensure_c3(a)
    lines = [l.split() for l in open(qlog).read().splitlines()]
    eng = w.VacuumEngine(idx, device=0, threads=16, positions=False)
    eng.Load()
    n_cu = 256   # MI355X (torch does not see the device from this process)
    bs = []
    for s in range(0, 8 * a.batch, a.batch):
        b = w.ResidentBatch(eng, a.batch, a.k)
        b.upload(bench.resolve(eng, lines[s:s + a.batch], a.k))
        bs.append(b)
    # the two-term instance's grid: 6 workgroups of 4 waves per CU (engine.cc lean_wgs_two)
    n_lean = n_cu * 6 * 4
    out = {"n_cu": n_cu, "alone": [], "pipelined": []}
    for b in bs:
        b.run()
        b.fetch()
        out["alone"].append(summary(rows(eng, b, n_lean)))
    for _ in range(3):
        for b in bs:
            b.run()
    w.sync(eng)
    for b in bs:
        out["pipelined"].append(summary(rows(eng, b, n_lean)))
    print(json.dumps(out))
    for b in bs:
        b.close()
    eng.close()


if __name__ == "__main__":
    main()
