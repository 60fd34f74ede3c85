#!/usr/bin/env python3
"""Per-class kernel times on the C3 stand-in (diagnostic, not the bench):
the C4 mix split by term count, the single-term groups, the headline's
two-term log and the realistic mix, each class as 4,096-query batches.  Per
class: one batch alone (plan / segment / lean HIP-event times, items, driver
blocks, survivors, algorithmic bytes) and the pipelined rate (two copies of
the batch in flight, like the bench's loop).

usage: diag_classes.py [CLASS ...]   (default: all)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    want = set(sys.argv[1:])
    sys.argv = [sys.argv[0], "--no-cpu"]
    a = bench.parse()
    import wiser_amd as w
    from wiser_amd import _capi
    idx, qlog, _ = bench.ensure_c3(a)
    mixed, _, _ = bench.leg_items(a, idx, "c4_mixed_1to5")
    classes = {"headline": [(l.split(), False) for l in open(qlog).read().splitlines()][:8192]}
    for n in range(1, 6):
        classes[f"c4_{n}term"] = [it for it in mixed if len(it[0]) == n]
    classes["c4_3to5"] = [it for it in mixed if len(it[0]) >= 3]
    classes["c4_mix"] = mixed
    for name in ("single_high", "single_low", "realistic_mix", "c5_phrase"):
        classes[name] = bench.leg_items(a, idx, name)[0]
    # the realistic mix's two parts alone (the same queries)
    classes["real_and"] = [it for it in classes["realistic_mix"] if not it[1]]
    classes["real_phrase"] = [it for it in classes["realistic_mix"] if it[1]]
    engs = {}
    for name, items in classes.items():
        if want and name not in want:
            continue
        items = items[:8192]
        if not items:
            continue
        ph = any(p for _, p in items)
        if ph not in engs:
            engs[ph] = w.VacuumEngine(idx, positions=ph)
            engs[ph].Load()
        eng = engs[ph]
        bs = []
        for s in range(0, len(items), 4096):
            chunk = items[s:s + 4096]
            arr = (_capi.Query * len(chunk))()
            for i, (t, p) in enumerate(chunk):
                arr[i] = eng.resolve(w.SearchQuery(t, n_results=10, is_phrase=p))[0]
            b = w.ResidentBatch(eng, len(chunk), 10)
            b.upload(arr)
            bs.append(b)
        for b in bs:
            b.run()
        w.sync(eng)
        alone = []
        for b in bs:
            b.run()
            b.fetch()
            alone.append(b.stats())
        n = 200
        w.sync(eng)
        t0 = time.perf_counter()
        for i in range(n):
            bs[i % len(bs)].run()
        w.sync(eng)
        el = (time.perf_counter() - t0) / n * 1e3
        st = alone[0]
        nq = sum(b.nq for b in bs) / len(bs)
        print(f"{name:14s} q/batch={nq:.0f} alone: plan={st.plan_ms:.3f} seg={st.segment_ms:.3f} "
              f"lean={st.lean_ms:.3f} items={st.work_items} dblk={st.driver_blocks} surv={st.survivors} "
              f"oblk={st.other_blocks} algoMB={st.algo_bytes / 1e6:.1f} | pipelined {el:.4f} ms/batch "
              f"= {nq / el * 1e3 / 1e6:.2f} M q/s, {st.algo_bytes / (el * 1e-3) / 1e12:.3f} TB/s algo",
              flush=True)
        for b in bs:
            b.close()
    for e in engs.values():
        e.close()


if __name__ == "__main__":
    main()
