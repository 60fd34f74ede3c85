#!/usr/bin/env python3
"""Per-query cost of the event replay on the high x high class (diagnostics:
needs the -DWSR_REPLAY_PROF build, make variant V=replayprof, loaded through
WISER_HIP_LIB).  Runs one batch's segments (events only), then the unfused
replay_kernel with per-query cycle counters, and prints how the replay time
relates to events, filter candidates and heap insertions.
Usage: replay_profile.py [--wiki]"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import wiser_amd as w  # noqa: E402
from wiser_amd import _capi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--wiki", action="store_true")
args = ap.parse_args()
idx = "/tmp/wiser_bench/c3_wiki_5500000_1" if args.wiki else "/tmp/wiser_bench/c2_1000000_500000"
if not os.path.exists(os.path.join(idx, "READY")):
    os.makedirs(idx, exist_ok=True)
    (w.build_wiki_standin if args.wiki else w.build_synthetic)(idx, threads=16)
    w.gen_two_term_log(idx, os.path.join(idx, "two_term_100000.log"), 100000, 7)
    open(os.path.join(idx, "READY"), "w").write("ok")
eng = w.VacuumEngine(idx, positions=False)
eng.Load()
lines = [l.split() for l in open(os.path.join(idx, "two_term_100000.log")).read().splitlines()]
hh = [t for t in lines if all(eng.lookup(x)[1] >= 10000 for x in t)][:4096]
b = w.ResidentBatch(eng, len(hh), 10)
b.upload(__import__("bench").resolve(eng, hh, 10))
_capi.check(_capi.lib.wsr_batch_run_events(eng._h, b._b))
rows = (C.c_uint32 * (6 * len(hh)))()
_capi.check(_capi.lib.wsr_debug_replay_profile(eng._h, b._b, rows))
r = np.frombuffer(rows, dtype=np.uint32).reshape(-1, 6).astype(np.int64)
filt, fin, ev, cand, ins, items = r.T
tot = filt + fin
print(f"{'C3' if args.wiki else 'C2'} high x high, {len(hh)} queries (s_memtime: core clock cycles)")
for name, v in (("filter", filt), ("finish", fin), ("total", tot), ("events", ev), ("candidates", cand),
                ("insertions", ins), ("items", items)):
    print(f"  {name:10s} mean {v.mean():10.1f} p50 {np.median(v):10.1f} p99 {np.percentile(v, 99):10.1f} "
          f"max {v.max():10d}")
for c in ("events", "candidates", "insertions"):
    x = {"events": ev, "candidates": cand, "insertions": ins}[c]
    print(f"  corr(total, {c}) = {np.corrcoef(tot, x)[0, 1]:.3f}")
top = np.argsort(-tot)[:8]
print("  slowest: ticks / events / candidates / insertions / items")
for i in top:
    print(f"    {tot[i]:8d} {ev[i]:6d} {cand[i]:6d} {ins[i]:6d} {items[i]:4d}")
b.close()
eng.close()
