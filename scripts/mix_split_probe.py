"""How a mixed batch (10 % two-term phrases among the 1-5-term AND mix,
bench.py's realistic_mix leg) should run: the leg's batches as they are,
each batch split by class into a conjunctive and a phrase sub-batch (what a
host-side split would submit), and the log sorted by class (pure batches).
Same timed loop as bench.run_leg (16+ batches resident, every batch run in
turn, consecutive batches in flight); prints one JSON line per form.

usage: mix_split_probe.py [PASSES]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    sys.argv = [sys.argv[0], "--no-cpu"]
    a = bench.parse()
    import wiser_amd as w
    from wiser_amd import _capi
    idx, _, _ = bench.ensure_c3(a)
    items, _, _ = bench.leg_items(a, idx, "realistic_mix")
    eng = w.VacuumEngine(idx, device=0, threads=bench.HOST_THREADS, positions=True)
    eng.Load()
    B = a.batch

    def batches_of(groups):
        out = []
        for g in groups:
            arr = (_capi.Query * len(g))()
            for i, (t, ph) in enumerate(g):
                arr[i] = eng.resolve(w.SearchQuery(t, n_results=a.k, is_phrase=ph))[0]
            b = w.ResidentBatch(eng, max(len(g), 1), a.k)
            b.upload(arr)
            out.append(b)
        return out

    chunks = [items[s:s + B] for s in range(0, len(items), B)]
    while len(chunks) < 16:
        chunks = chunks + chunks
    chunks = chunks[:16]
    forms = {
        "mixed": chunks,
        "split": [g for c in chunks for g in ([x for x in c if not x[1]], [x for x in c if x[1]]) if g],
        "sorted": (lambda flat: [flat[s:s + B] for s in range(0, len(flat), B)])(
            sorted([x for c in chunks for x in c], key=lambda x: x[1])),
    }
    for name, groups in forms.items():
        bs = batches_of(groups)
        nq = sum(len(g) for g in groups)
        for b in bs:
            b.run()
        w.sync(eng)
        t0 = time.perf_counter()
        for _ in range(passes):
            for b in bs:
                b.run()
        w.sync(eng)
        el = time.perf_counter() - t0
        for b in bs:
            b.fetch()
            b.close()
        print(json.dumps({"form": name, "value": round(nq * passes / el, 1), "batches": len(bs),
                          "queries_per_pass": nq, "ms_per_pass": round(el / passes * 1e3, 4)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
