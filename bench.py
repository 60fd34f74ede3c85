#!/usr/bin/env python3
"""Throughput bench: 2-term AND + BM25 top-10 over a Vacuum index on MI355X.

Workload (BASELINE.json configs[1], SURVEY.md 8d "C2"): 1M synthetic Zipf docs
(V=500k, s=1.07, lognormal lengths, seed 0x5EED2026) written in the reference's
Vacuum layout by the build's writer; 100k two-term queries drawn by the
gen_synthetic_log.py:191-214 rule (seed 7); batches of 4096 queries; k = 10.
The English-Wikipedia index of configs[2..4] is not available offline.

A step = one batch (4096 queries per GPU) through plan + segment + replay
kernels, with the batch's resolved queries already resident in HBM.
value = queries completed by all ranks / max-over-ranks wall time.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "queries/sec + p50 lat, 2-term AND BM25 top-10 on Wikipedia, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=25)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--docs", type=int, default=1_000_000)
    p.add_argument("--vocab", type=int, default=500_000)
    p.add_argument("--queries", type=int, default=100_000)
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--index-dir", default=os.environ.get("WISER_BENCH_DIR", "/tmp/wiser_bench"))
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="bounded CPU-baseline sample (oracle, 1 thread), rank 0 at N=1")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--check", type=int, default=256, help="queries checked against the oracle")
    return p.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # gloo for the control plane (barrier, max)
        dist.init_process_group("gloo")

    import wiser_amd as w
    from wiser_amd import _capi

    idx = os.path.join(a.index_dir, f"c2_{a.docs}_{a.vocab}")
    qlog = os.path.join(idx, f"two_term_{a.queries}.log")
    if rank == 0 and not os.path.exists(os.path.join(idx, "READY")):
        os.makedirs(idx, exist_ok=True)
        t = time.time()
        st = w.build_synthetic(idx, n_docs=a.docs, vocab=a.vocab, threads=min(16, os.cpu_count()))
        w.gen_two_term_log(idx, qlog, n_queries=a.queries, seed=7)
        open(os.path.join(idx, "READY"), "w").write("ok")
        log(f"built index {st.n_docs} docs {st.n_terms} terms {st.n_postings} postings "
            f"{st.vacuum_bytes/1e9:.2f} GB in {time.time()-t:.1f}s")
    if dist:
        dist.barrier()

    t = time.time()
    eng = w.VacuumEngine(idx, device=local, threads=min(16, os.cpu_count()))
    eng.Load()
    log(f"rank {rank}: engine loaded in {time.time()-t:.1f}s")

    lines = [l.split() for l in open(qlog).read().splitlines()]
    # each rank serves its own replica slice of the log (independent queries)
    per_rank = (len(lines) + world - 1) // world
    mine = lines[rank * per_rank:(rank + 1) * per_rank] or lines[:a.batch]
    batches = []
    for s in range(0, len(mine), a.batch):
        chunk = mine[s:s + a.batch]
        arr = (_capi.Query * len(chunk))()
        for i, terms in enumerate(chunk):
            q, _ = eng.resolve(w.SearchQuery(terms, n_results=a.k))
            arr[i] = q
        b = w.ResidentBatch(eng, a.batch, a.k)
        b.upload(arr)
        batches.append((b, chunk))
    nb = len(batches)

    # correctness spot-check against the oracle (checker only)
    checked = 0
    if a.check and rank == 0:
        from oracle.oracle import OracleVacuum
        orc = OracleVacuum(idx)
        b, chunk = batches[0]
        b.run()
        hits, nh = b.fetch()
        for i, terms in enumerate(chunk[:a.check]):
            want, _ = orc.search(terms, a.k)
            got = [(hits[i * a.k + j].doc_id, hits[i * a.k + j].score) for j in range(nh[i])]
            if got != want:
                raise SystemExit(f"parity failure on {terms}: {got[:3]} vs {want[:3]}")
            checked += 1
        orc.close()

    for s in range(a.warmup):
        batches[s % nb][0].run()
    w.sync(eng)

    # per-batch latency (each batch alone, submit -> results on the host)
    lat = []
    for b, _ in batches:
        t0 = time.perf_counter()
        b.run()
        b.fetch()
        lat.append((time.perf_counter() - t0) * 1e3)
    p50 = statistics.median(lat)

    if dist:
        dist.barrier()
    w.sync(eng)
    t0 = time.perf_counter()
    for s in range(a.steps):
        batches[s % nb][0].run()
    w.sync(eng)
    el = time.perf_counter() - t0
    queries = sum(batches[s % nb][0].nq for s in range(a.steps))

    # kernel-level accounting over one pass of the batches (HIP events on the engine stream)
    seg_ms = plan_ms = rep_ms = 0.0
    algo = surv = dblk = oblk = items = 0
    for b, _ in batches:
        b.run()
        w.sync(eng)
        st = b.stats()
        seg_ms += st.segment_ms
        plan_ms += st.plan_ms
        rep_ms += st.replay_ms
        algo += st.algo_bytes
        surv += st.survivors
        dblk += st.driver_blocks
        oblk += st.other_blocks
        items += st.work_items
    seg_avg_ms = seg_ms / nb
    achieved = (algo / nb) / (seg_avg_ms * 1e-3) / 1e9

    if dist:
        import torch
        tt = torch.tensor([el, float(queries)], dtype=torch.float64)
        mx = tt.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tt.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        el, queries = mx[0].item(), sm[1].item()
    qps = queries / el

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        from oracle.oracle import OracleVacuum
        orc = OracleVacuum(idx)
        done, t0 = 0, time.perf_counter()
        step = 64
        while time.perf_counter() - t0 < a.cpu_seconds and done < len(lines):
            orc.search_lines(lines[done:done + step], a.k, threads=1)
            done += step
        cel = time.perf_counter() - t0
        orc.close()
        cpu = {"value": round(done / cel, 1), "unit": "queries/s", "cores": 1, "kind": "port",
               "sample": f"first {done} queries of the same log, oracle restatement of "
                         f"VacuumEngine::Search, 1 thread, {cel:.1f}s"}

    traffic = None
    pmc = os.path.join(ROOT, "profiles", "r01_pmc_segment.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(qps, 1), "unit": "queries/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32/f64",
            "data": "synthetic",
            "config": {"workload": f"C2: {a.docs} synthetic Zipf docs (V={a.vocab}, s=1.07), "
                                   f"{len(lines)} two-term AND queries (gen_synthetic_log rule, "
                                   f"seed 7), batch {a.batch}, top-{a.k}",
                       "global_batch": a.batch * world, "parallelism": f"replicas{world}",
                       "k": a.k},
            "p50_ms": round(p50, 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel": "segment_kernel", "algo_bytes_per_launch": int(algo / nb),
                         "avg_launch_ms": round(seg_avg_ms, 4)},
            "cpu_baseline": cpu,
            "kernel_ms_per_batch": {"plan": round(plan_ms / nb, 4), "segment": round(seg_avg_ms, 4),
                                    "replay": round(rep_ms / nb, 4)},
            "per_batch": {"survivors": int(surv / nb), "driver_blocks": int(dblk / nb),
                          "other_blocks": int(oblk / nb), "work_items": int(items / nb)},
            "parity_checked_queries": checked,
        }
        print(json.dumps(out), flush=True)
    for b, _ in batches:
        b.close()
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
