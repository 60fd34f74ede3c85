#!/usr/bin/env python3
"""A/B of the GPU phrase path with and without the two-way bloom filters
(bloom_enable_factor 1 vs 0, query_processing.h:873-884) on a natural-text
positions index written WITH blooms by the streaming writer.

The C5 stand-in's lists are drawn per term (no per-doc token sequence), so it
has no neighbour filters; this index is a Zipf token stream (make_linedoc.py
WITH_POSITIONS), so its phrase queries are real adjacent bigrams of the
corpus, as the reference's phrase pool (gen_synthetic_log.py:216-265).

usage: phrase_bloom_ab.py WORK_DIR [n_docs] [n_queries] > ab.json"""
import json
import os
import random
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    work = sys.argv[1]
    n_docs = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
    nq = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
    os.makedirs(work, exist_ok=True)
    import wiser_amd as w
    import bench
    ld = os.path.join(work, f"zipf_pos_{n_docs}.linedoc")
    t = time.time()
    if not os.path.exists(ld):
        subprocess.check_call([sys.executable, os.path.join(ROOT, "scripts", "make_linedoc.py"), ld, str(n_docs),
                               "WITH_POSITIONS", "3"])
    gen_s = time.time() - t
    idx = os.path.join(work, f"zipf_pos_{n_docs}_bloom")
    t = time.time()
    if not os.path.exists(os.path.join(idx, "my.vacuum")):
        st = w.build_from_linedoc(ld, idx, "WITH_POSITIONS", bloom=(0.0009, 5))
    build_s = time.time() - t
    # bigram phrase log: adjacent tokens of random docs (phrase-pool style)
    rng = random.Random(7)
    want = set(rng.sample(range(n_docs), min(n_docs, nq)))
    qs = []
    with open(ld) as f:
        f.readline()
        for d, line in enumerate(f):
            if d in want:
                toks = line.split("\t")[1].split()
                i = rng.randrange(len(toks) - 1)
                if toks[i] != toks[i + 1]:
                    qs.append([toks[i], toks[i + 1]])
    items = [(q, True) for q in qs]
    out = {"index": os.path.basename(idx), "n_docs": n_docs, "linedoc_gen_s": round(gen_s, 1),
           "index_build_s": round(build_s, 1), "queries": len(items),
           "workload": "two-term phrase queries = adjacent token pairs of random docs, top-10", "runs": {}}
    for factor in (0, 1, 0, 1):
        eng = w.VacuumEngine(idx, bloom_factor=factor, positions=True)
        t = time.time()
        eng.Load()
        load_s = time.time() - t
        leg = bench.run_leg(eng, idx, items, 10, 4096, 8, 128, 0)
        leg["load_s"] = round(load_s, 1)
        leg["image_pos_bytes"] = eng.image_info()["pos_bytes"]
        eng.close()
        key = f"bloom_factor_{factor}"
        out["runs"].setdefault(key, []).append({k: leg[k] for k in (
            "value", "ms_per_batch", "p50_alone_ms", "segment_ms_per_batch", "survivors_per_batch",
            "parity_checked_queries", "load_s", "image_pos_bytes")})
        print(key, leg["value"], leg["segment_ms_per_batch"], file=sys.stderr)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
