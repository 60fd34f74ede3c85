#!/usr/bin/env python3
"""Per-query-class kernel times on the C2 index (diagnostic, not the bench)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import wiser_amd as w
from wiser_amd import _capi

import argparse
ap = argparse.ArgumentParser()
ap.add_argument("--index", default="/tmp/wiser_bench/c2_1000000_500000")
ap.add_argument("--only", default="")
ap.add_argument("--repeat", type=int, default=1)
ap.add_argument("--wiki", action="store_true", help="the C3 stand-in (bench.py c3_leg's index)")
args = ap.parse_args()
if args.wiki and args.index == ap.get_default("index"):
    args.index = "/tmp/wiser_bench/c3_wiki_5500000_1"
idx = args.index
if not os.path.exists(os.path.join(idx, "READY")):
    os.makedirs(idx, exist_ok=True)
    if args.wiki:
        w.build_wiki_standin(idx, threads=16)
    else:
        w.build_synthetic(idx, threads=16)
    w.gen_two_term_log(idx, os.path.join(idx, "two_term_100000.log"), 100000, 7)
    open(os.path.join(idx, "READY"), "w").write("ok")
eng = w.VacuumEngine(idx, positions=False)
eng.Load()
lines = [l.split() for l in open(os.path.join(idx, "two_term_100000.log")).read().splitlines()]
cls = {"mixed": lines[:4096], "low-low": [], "low-high": [], "high-high": [],
       "hh-lean": [], "hh-general": []}
n_docs = eng.NumDocs()
for t in lines:
    dfs = [eng.lookup(x)[1] for x in t]
    h = sum(1 for d in dfs if d >= 10000)
    cls[["low-low", "low-high", "high-high"][h]].append(t)
    if h == 2:   # the other (longer) list has a rank bitmap: df >= N / 128 (WSR_DENSE_DIV)
        cls["hh-lean" if max(dfs) * 128 >= n_docs else "hh-general"].append(t)
import ctypes as C
for name, qs in cls.items():
    if args.only and name != args.only:
        continue
    qs = qs[:4096]
    if not qs:
        print(f"{name:10s} n=0")
        continue
    arr = (_capi.Query * len(qs))()
    for i, t in enumerate(qs):
        arr[i] = eng.resolve(w.SearchQuery(t, n_results=10))[0]
    b = w.ResidentBatch(eng, len(qs), 10)
    b.upload(arr)
    for _ in range(3):
        b.run()
    w.sync(eng)
    for _ in range(args.repeat):
        b.run()
    st = b.stats()
    print(f"{name:10s} n={len(qs)} plan={st.plan_ms:.3f} seg={st.segment_ms:.3f} lean={st.lean_ms:.3f} "
          f"replay={st.replay_ms:.3f} "
          f"items={st.work_items} surv={st.survivors} dblk={st.driver_blocks} oblk={st.other_blocks} "
          f"algoMB={st.algo_bytes/1e6:.1f} events={st.events} maxqev={st.max_query_events}", flush=True)
    n_wg, stride = C.c_int32(), C.c_int32()
    _capi.check(_capi.lib.wsr_debug_wg_stats(eng._h, b._b, None, 0, C.byref(n_wg), C.byref(stride)))
    raw = (C.c_uint32 * (n_wg.value * stride.value))()
    _capi.check(_capi.lib.wsr_debug_wg_stats(eng._h, b._b, raw, len(raw), None, None))
    rows = [raw[i * stride.value:(i + 1) * stride.value] for i in range(n_wg.value)]
    db = sorted(r[1] for r in rows)
    print(f"   wg={n_wg.value} driver blocks per wg: mean={sum(db)/len(db):.1f} max={db[-1]} "
          f"p50={db[len(db)//2]} p99={db[int(len(db)*0.99)]}")
    if stride.value >= 10:
        names = (["setup", "driver", "dense", "blocks", "topk"] if os.environ.get("WSR_DIAG_GENERAL")
                 else ["setup", "segment", "finish", "dequeue", "-"])
        tot = [sum(r[4 + i] for r in rows) for i in range(5)]
        wall = sorted(r[9] for r in rows)
        allc = sum(tot)
        print("   sections: " + " ".join(f"{n}={100*t/allc:.1f}%" for n, t in zip(names, tot)) +
              f" | wg cycles mean={sum(wall)/len(wall):.0f} p50={wall[len(wall)//2]} max={wall[-1]}"
              f" | cycles/driver block={allc/max(1,sum(db)):.0f}")
        if not os.environ.get("WSR_DIAG_GENERAL"):
            st = [sum(r[10 + i] for r in rows) for i in range(4)]
            print("   lean stages per driver block: " +
                  " ".join(f"{n}={t/max(1,sum(db)):.0f}" for n, t in zip("WCHD", st)))
    b.close()
print("class sizes:", {k: len(v) for k, v in cls.items()})
