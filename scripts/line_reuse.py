"""Cache-line reuse of the lean kernel's bitmap probes across one batch
(CPU estimate, diagnostics only).

For the first BATCH two-term queries of a log whose other list carries a rank
bitmap (df >= span / 2048), every driver posting probes O1's bitmap (8 B per 32
docs: a 128-byte line covers 512 docs).  Reports, per driver block, the lines
one query touches (its own distinct lines, what the kernel fetches when no
line is shared with another query) and, over the batch, how many of those
fetches are of a line that another query of the batch also probes (what an L2
could serve if the queries sharing an O1 list ran on one XCD at once), plus
the same for a 1-bit presence bitmap (1,024 docs per line).

usage: line_reuse.py INDEX_DIR LOG [BATCH]"""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from oracle.oracle import OracleVacuum
    idx, log = sys.argv[1], sys.argv[2]
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    o = OracleVacuum(idx)
    n_docs = 5_500_000
    dense_df = n_docs // 2048
    cache = {}

    def plist(t):
        if t not in cache:
            cache[t] = np.asarray(o.postings(t)[0], dtype=np.int64)
        return cache[t]

    lines = [l.split() for l in open(log).read().splitlines()][:batch]
    per_query = []          # (o1 term, set of 512-doc lines, set of 1024-doc lines, driver blocks)
    n_general = 0
    for t in lines:
        if len(t) != 2 or o.df(t[0]) == 0 or o.df(t[1]) == 0:
            continue
        a, b = plist(t[0]), plist(t[1])
        drv, oth, ot = (a, b, t[1]) if len(a) <= len(b) else (b, a, t[0])
        if len(oth) < dense_df:
            n_general += 1
            continue
        per_query.append((ot, np.unique(drv // 512), np.unique(drv // 1024), (len(drv) + 127) // 128))
    blocks = sum(q[3] for q in per_query)
    for name, col in (("2-bit rank bitmap (512 docs/line)", 1), ("1-bit bitmap (1024 docs/line)", 2)):
        total = sum(len(q[col]) for q in per_query)
        uses = collections.Counter()
        for q in per_query:
            for x in q[col].tolist():
                uses[(q[0], x)] += 1
        distinct = len(uses)
        shared = sum(c for c in uses.values() if c > 1)
        print(f"{name}: {len(per_query)} lean queries, {blocks} driver blocks; "
              f"lines fetched per query (distinct within the query) {total} = {total / blocks:.1f} per block; "
              f"distinct over the batch {distinct} ({distinct / blocks:.1f} per block); "
              f"fetches of a line another query also probes {shared} ({100 * shared / total:.1f} %)")
    o1 = collections.Counter(q[0] for q in per_query)
    top = o1.most_common(10)
    print(f"general-kernel queries: {n_general}; distinct O1 lists {len(o1)}; most common O1: "
          + ", ".join(f"{t}x{c}" for t, c in top))


if __name__ == "__main__":
    main()
