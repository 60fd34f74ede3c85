"""Where a C3 headline launch's L2-miss traffic comes from, by source (CPU
model, diagnostics only; the counters give only the total).

For the first BATCH two-term queries of a log it restates the plan's class
rule (an other list with a rank bitmap -- df >= span / 2048 -- makes the query
lean) and counts, per query, the distinct 128-byte lines each source reads
when no line is shared with another query and nothing is pruned:
  driver   the driver's doc-id and tf packs (bit widths from the block's
           largest delta / tf), its plen line and directory entries (lean);
  mask     O1's 4-byte mask words, one per probed driver posting inside O1's
           doc range (1,024 docs per line);
  rank     the 8-byte rank records of the hits (512 docs per line);
  tf8      O1's tf bytes read by rank, for hits past a word's fourth posting;
  general  (general class) the other list's packs of every block whose doc
           range holds a driver posting, plus the driver's packs;
  events   16 B per survivor written and read back (an upper bound: the
           running top-k keeps far fewer);
and the algorithmic bytes of bench.py's rule (each term's docid + tf pack
bytes, + 1 B per survivor + 12 B per result).  Pruned runs probe fewer
postings: the survivors the GPU reports per batch (bench.py
`survivors_per_batch`) against the model's hits scale the hit-side sources.

usage: traffic_model.py INDEX_DIR LOG [BATCH] [FIRST]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LINE = 128


def nlines(addrs):
    return len(np.unique(np.asarray(addrs, dtype=np.int64) // LINE)) if len(addrs) else 0


def pack_bytes(docs, tfs):
    """Per 128-posting block: docid pack + tf pack bytes (full blocks), VInts
    bytes for the last partial block (as the file stores them)."""
    n = len(docs)
    out = []
    gaps = np.diff(np.concatenate([[0], docs]))
    for s in range(0, n, 128):
        g, t = gaps[s:s + 128], tfs[s:s + 128]
        if len(g) == 128:
            bd = int(max(1, int(g.max()).bit_length()))
            bt = int(max(1, int(t.max()).bit_length()))
            out.append(16 * bd + 16 * bt + 4)
        else:
            vb = lambda a: int(np.sum((np.asarray(a) >= 128) + (np.asarray(a) >= 16384) + 1))
            out.append(vb(g) + vb(t))
    return np.asarray(out, dtype=np.int64)


def main():
    from oracle.oracle import OracleVacuum
    idx, log = sys.argv[1], sys.argv[2]
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    first = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    o = OracleVacuum(idx)
    n_docs = o.n_docs()
    dense_df = n_docs // 2048
    cache = {}

    def plist(t):
        if t not in cache:
            d, tf = o.postings(t)
            d = np.asarray(d, dtype=np.int64)
            tf = np.asarray(tf, dtype=np.int64)
            cache[t] = (d, tf, pack_bytes(d, tf))
        return cache[t]

    qs = [l.split() for l in open(log).read().splitlines()][first:first + batch]
    src = dict(driver=0, mask=0, rank=0, tf8=0, general=0, events=0)
    algo = 0
    cls = dict(lean=0, general=0, empty=0)
    hits_tot = 0
    by_df = {}   # driver df decade -> [queries, lines, algo]
    for t in qs:
        if len(t) != 2 or o.df(t[0]) == 0 or o.df(t[1]) == 0:
            cls["empty"] += 1
            continue
        a, b = plist(t[0]), plist(t[1])
        (dd, dtf, dpb), (od, otf, opb) = (a, b) if len(a[2]) <= len(b[2]) else (b, a)
        qa = int(dpb.sum() + opb.sum()) + 120
        hit = np.isin(dd, od)
        nh = int(hit.sum())
        qa += nh
        algo += qa
        hits_tot += nh
        ql = 0
        # the driver's packs, plen and directory (every block)
        drv_lines = int(np.sum((dpb + LINE - 1) // LINE)) + len(dpb) + (len(dpb) * 20 + LINE - 1) // LINE
        ql += drv_lines
        src["driver"] += drv_lines
        if len(od) >= dense_df:
            cls["lean"] += 1
            inr = dd[(dd >= 0) & (dd <= od[-1])]
            m = nlines((inr // 32) * 4)
            hd = dd[hit]
            r = nlines((hd // 32) * 8)
            # O1 rank of each hit and its index within its 32-doc word
            rk = np.searchsorted(od, hd)
            w0 = np.searchsorted(od, (hd // 32) * 32)
            esc = rk[(rk - w0) >= 4]
            f = nlines(esc)
            src["mask"] += m
            src["rank"] += r
            src["tf8"] += f
            ql += m + r + f
        else:
            cls["general"] += 1
            ob = np.searchsorted(od[127::128] if len(od) >= 128 else od[-1:], dd)
            ob = np.unique(np.minimum(ob, len(opb) - 1))
            g = int(np.sum((opb[ob] + LINE - 1) // LINE))
            src["general"] += g
            ql += g
        ev = (nh * 16 * 2 + LINE - 1) // LINE
        src["events"] += ev
        ql += ev
        dec = int(np.log10(max(1, len(dd))))
        e = by_df.setdefault(dec, [0, 0, 0])
        e[0] += 1
        e[1] += ql
        e[2] += qa
    tot = sum(src.values())
    print(f"{idx}: queries {first}..{first + len(qs)} of {log}: classes {cls}, hits {hits_tot}")
    print(f"algorithmic bytes {algo / 1e6:.1f} MB; modelled lines {tot} = {tot * LINE / 1e6:.1f} MB "
          f"({tot * LINE / max(1, algo):.2f}x algorithmic), no pruning, no line shared between queries")
    for k, v in src.items():
        print(f"  {k:8s} {v:9d} lines {v * LINE / 1e6:8.1f} MB  {100 * v / max(1, tot):5.1f} %")
    print("by driver df decade (queries, modelled MB, algorithmic MB, ratio):")
    for dec in sorted(by_df):
        q, l, a_ = by_df[dec]
        print(f"  1e{dec}: {q:5d} {l * LINE / 1e6:8.1f} {a_ / 1e6:8.1f} {l * LINE / max(1, a_):6.2f}")
    o.close()


if __name__ == "__main__":
    main()
