#!/usr/bin/env python3
"""How often a C3 headline query's top-(k+1) holds a score tie (diagnostic):
the replay's heap order matters only among equal scores.  Runs the first
8 batches of the headline log at k+1 = 11 and prints, over all queries and
over those with the most driver blocks (heavy: the batch tail's replays), the
share whose 11 best scores are not all distinct."""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import bench  # noqa: E402
import wiser_amd as w  # noqa: E402


def main():
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    idx, qlog, _ = bench.ensure_c3(a)
    lines = [l.split() for l in open(qlog).read().splitlines()][:8 * a.batch]
    eng = w.VacuumEngine(idx, device=0, threads=16, positions=False)
    eng.Load()
    k1 = 11
    res = []
    for s in range(0, len(lines), a.batch):
        chunk = lines[s:s + a.batch]
        b = w.ResidentBatch(eng, len(chunk), k1)
        b.upload(bench.resolve(eng, chunk, k1))
        b.run()
        hits, nh = b.fetch()
        for i, q in enumerate(chunk):
            n = nh[i]
            sc = [hits[i * k1 + j].score for j in range(n)]
            res.append((n, len(set(sc)) < n))
        b.close()
    # heavy: the queries whose shorter list is longest (document frequency)
    dfs = []
    for q in lines:
        f = eng.resolve(w.SearchQuery(q, n_results=k1))[1]
        dfs.append(min(f) if f else 0)
    out = {"queries": len(res), "tie_share": round(sum(t for _, t in res) / len(res), 4),
           "full_share": round(sum(n == k1 for n, _ in res) / len(res), 4)}
    if dfs:
        order = sorted(range(len(res)), key=lambda i: -dfs[i])[:len(res) // 20]
        out["heavy5pct_tie_share"] = round(sum(res[i][1] for i in order) / len(order), 4)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
