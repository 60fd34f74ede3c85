#!/usr/bin/env python3
"""Per-GPU cost of doc-range sharding at world size W, simulated on one GPU:
shard r of W runs a global batch of 4096*W queries (plan+segment+reduce+pack)."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import wiser_amd as w
from wiser_amd import _capi
from wiser_amd._capi import check, lib
from wiser_amd.shard import index_doc_count, shard_range

idx = "/tmp/wiser_bench/c2_1000000_500000"
if not os.path.exists(os.path.join(idx, "READY")):
    os.makedirs(idx, exist_ok=True)
    w.build_synthetic(idx, threads=16)
    w.gen_two_term_log(idx, os.path.join(idx, "two_term_100000.log"), 100000, 7)
    open(os.path.join(idx, "READY"), "w").write("ok")
lines = [l.split() for l in open(os.path.join(idx, "two_term_100000.log")).read().splitlines()]
n = index_doc_count(idx)
for W in (1, 2, 4, 8):
    for r in (0, W - 1):
        e = w.VacuumEngine(idx, doc_range=shard_range(n, r, W) if W > 1 else None, threads=16)
        e.Load()
        Q = 4096 * W
        arr = (_capi.Query * Q)()
        for i in range(Q):
            arr[i] = e.resolve(w.SearchQuery(lines[i], n_results=10))[0]
        b = w.ResidentBatch(e, Q, 10)
        b.upload(arr)
        cnt = torch.empty(Q, dtype=torch.int32, device="cuda")
        tot = (C.c_int64 * W)()
        for it in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            check(lib.wsr_batch_run_events(e._h, b._b) if W > 1 else lib.wsr_batch_run(e._h, b._b))
            w.sync(e)
            t1 = time.perf_counter()
            check(lib.wsr_shard_reduce(e._h, b._b, 4096, W, C.c_void_p(cnt.data_ptr()), tot))
            send = torch.empty((max(sum(tot), 1), 2), dtype=torch.int64, device="cuda")
            check(lib.wsr_shard_pack(e._h, b._b, C.c_void_p(send.data_ptr())))
            t2 = time.perf_counter()
        st = b.stats()
        print(f"W={W} shard={r} Q={Q} run={1e3*(t1-t0):.3f}ms (plan {st.plan_ms:.3f} seg {st.segment_ms:.3f} "
              f"replay {st.replay_ms:.3f}) reduce+pack={1e3*(t2-t1):.3f}ms events={sum(tot)} "
              f"({sum(tot)*16/1e6:.1f} MB) items={st.work_items}", flush=True)
        b.close()
        e.close()
