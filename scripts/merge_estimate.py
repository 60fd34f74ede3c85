"""Cache lines a high x high query touches per driver block, bitmap probe vs
merge (CPU estimate over an index and its two-term log).

Bitmap path (lean_kernel): every driver posting probes O1's rank bitmap (8 B
per 32 docs, so one 128-byte line covers 512 docs) and every hit gathers one
tf byte of O1's tf8 array (one line per 128 ranks).  Merge path: the O1 blocks
whose doc range overlaps the driver block are read whole (doc-id pack ~ 16 b
bytes, b bits per value, plus the 128 tf bytes of tf8).  Both add the driver's
own pack and length-code lines, left out here.

usage: merge_estimate.py INDEX_DIR LOG [n_queries]"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from oracle.oracle import OracleVacuum
    idx, log = sys.argv[1], sys.argv[2]
    nq = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    o = OracleVacuum(idx)
    qs = []
    for line in open(log):
        t = line.split()
        if len(t) == 2 and min(o.df(t[0]), o.df(t[1])) >= 10000:
            qs.append(t)
        if len(qs) >= nq:
            break
    tot = dict(blocks=0, bm_lines=0, tf_lines=0, o1_blocks=0, merge_lines=0, probes=0, hits=0)
    ratio_hist = {}
    for a, b in qs:
        da, _ = o.postings(a)
        db, _ = o.postings(b)
        drv, oth = (da, db) if len(da) <= len(db) else (db, da)
        r = len(oth) / len(drv)
        key = "<=1.5" if r <= 1.5 else "<=2" if r <= 2 else "<=4" if r <= 4 else "<=8" if r <= 8 else ">8"
        ratio_hist[key] = ratio_hist.get(key, 0) + 1
        rank = {d: i for i, d in enumerate(oth)}
        o_last = [oth[min(len(oth) - 1, i + 127)] for i in range(0, len(oth), 128)]
        o_first = [oth[i] for i in range(0, len(oth), 128)]
        # O1 pack width per block ~ bits of its largest gap
        o_bits = []
        for i in range(0, len(oth), 128):
            blk = oth[i:i + 128]
            prev = oth[i - 1] if i else 0
            g = max(x - y for x, y in zip(blk, [prev] + blk[:-1]))
            o_bits.append(max(1, g.bit_length()))
        j0 = 0
        for i in range(0, len(drv), 128):
            blk = drv[i:i + 128]
            lo, hi = blk[0], blk[-1]
            tot["blocks"] += 1
            tot["probes"] += len(blk)
            tot["bm_lines"] += len(set(d // 512 for d in blk))
            hit_ranks = [rank[d] for d in blk if d in rank]
            tot["hits"] += len(hit_ranks)
            tot["tf_lines"] += len(set(x // 128 for x in hit_ranks))
            while j0 < len(o_last) and o_last[j0] < lo:
                j0 += 1
            j = j0
            while j < len(o_first) and o_first[j] <= hi:
                tot["o1_blocks"] += 1
                tot["merge_lines"] += math.ceil(16 * o_bits[j] / 128) + 1 + 1   # pack (+1 misaligned) + tf8
                j += 1
    n = max(1, tot["blocks"])
    print(f"index {os.path.basename(idx.rstrip('/'))}: {len(qs)} high x high queries, {tot['blocks']} driver blocks")
    print("O1 / driver length:", dict(sorted(ratio_hist.items())))
    print(f"per driver block: bitmap lines {tot['bm_lines'] / n:.1f}, tf8 lines {tot['tf_lines'] / n:.1f} "
          f"(probe path {(tot['bm_lines'] + tot['tf_lines']) / n:.1f}); O1 blocks overlapped {tot['o1_blocks'] / n:.2f}, "
          f"merge lines {tot['merge_lines'] / n:.1f}; hits per block {tot['hits'] / n:.1f}")


if __name__ == "__main__":
    main()
