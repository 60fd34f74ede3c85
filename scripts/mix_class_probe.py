"""Probe: the realistic mix cut by the batch former as it is (conjunctive |
phrase) against a finer cut that also separates the conjunctive queries by
term count (two terms | one term | more), so that each batch runs the lean
instance of its class (kTwo / kOne / general).  One JSON line per form.

usage: mix_class_probe.py [PASSES]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    import bench
    sys.argv = [sys.argv[0], "--no-cpu"]
    a = bench.parse()
    import wiser_amd as w
    idx, _, _ = bench.ensure_c3(a)
    items, what, positions = bench.leg_items(a, idx, "realistic_mix")
    eng = w.VacuumEngine(idx, device=0, threads=bench.HOST_THREADS, positions=positions)
    eng.Load()
    base = w.class_batches

    def finer(queries, batch):
        order, nc = w.class_order(queries)
        conj = order[:nc]

        def cls(i):
            q = queries[i]
            if q.n_terms == 2 and q.k <= 64:
                return 0
            return 1 if q.n_terms == 1 else 2
        parts = [[i for i in conj if cls(i) == c] for c in range(3)] + [order[nc:]]
        out = []
        for p in parts:
            for s in range(0, len(p), batch):
                out.append(p[s:s + batch])
        return out

    for name, fn in (("conj_phrase", base), ("by_terms", finer), ("conj_phrase_2", base), ("by_terms_2", finer)):
        w.class_batches = fn
        out = bench.run_leg(eng, idx, items, a.k, a.batch, passes, 0, 0, class_form=True)
        print(json.dumps({"form": name, "value": out["value"], "ms_per_batch": out.get("ms_per_batch"),
                          "distinct_batches": out.get("distinct_batches")}), flush=True)
    w.class_batches = base
    eng.close()


if __name__ == "__main__":
    main()
