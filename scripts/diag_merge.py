"""Merge-class mismatches on the 20k synthetic index: for every query whose
top-k differs from the oracle's, the lists' sizes and the docs that differ.
Usage: python scripts/diag_merge.py [n_queries] [k]"""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    nq = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    import wiser_amd as w
    from oracle.oracle import OracleVacuum
    d = tempfile.mkdtemp(prefix="diag_merge_")
    w.build_synthetic(d, n_docs=20000, vocab=20000, seed=0x5EED2026, threads=4)
    log = os.path.join(d, "q.log")
    w.gen_two_term_log(d, log, n_queries=nq, seed=7)
    qs = [l.split() for l in open(log).read().splitlines()]
    os.environ.update({"WSR_MERGE_RATIO": "1000000000", "WSR_MERGE_MIN": "1"})
    eng = w.VacuumEngine(d)
    eng.Load()
    orc = OracleVacuum(d)
    res = eng.SearchBatch([w.SearchQuery(list(q), n_results=k) for q in qs])
    bad = 0
    for q, r in zip(qs, res):
        want, dfs = orc.search(list(q), k)
        got = [(e.doc_id, e.doc_score) for e in r.entries]
        same = len(got) == len(want) and all(g[0] == x[0] and abs(g[1] - x[1]) <= 1e-5 * max(1, abs(x[1]))
                                             for g, x in zip(got, want))
        if same:
            continue
        bad += 1
        if bad <= 12:
            full, _ = orc.search(list(q), 100000)
            gd = {x[0]: x[1] for x in got}
            wd = {x[0]: x[1] for x in want}
            fd = {x[0]: x[1] for x in full}
            print("query", q, "dfs", dfs, "n_hits", len(full))
            print("  got ", [(a, round(b, 5)) for a, b in got])
            print("  want", [(a, round(b, 5)) for a, b in want])
            print("  missing", sorted(set(wd) - set(gd)), "extra", [(x, round(gd[x], 5), x in fd) for x in sorted(set(gd) - set(wd))])
            print("  score diffs", [(x, round(gd[x], 5), round(wd[x], 5)) for x in gd if x in wd and abs(gd[x] - wd[x]) > 1e-5])
    print("bad", bad, "of", len(qs))


if __name__ == "__main__":
    main()
