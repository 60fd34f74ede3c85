#!/usr/bin/env python3
"""How many driver postings of the high x high class could a per-posting score
bound rule out before the other list is probed?  (Measurement only, CPU, numpy
over the oracle's decoded lists; the block-level form is blockmax_estimate.py.)

For a driver posting the driver's own BM25 part is exact (its tf and length
code are in hand before the probe); the other term's part is bounded by
  idf_o * tfn(M, norm(len))
with M the other list's largest tf (whole list, or its 2048-doc window).  A
posting whose bound is <= the threshold known before its block -- max(k-th
best of earlier segments, the segment's running k-th best) -- can hold no heap
insertion (the heap inserts only on a strictly larger score).
Usage: posting_bound_estimate.py INDEX_DIR LOG [N_QUERIES]"""
import struct
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from oracle.oracle import OracleVacuum  # noqa: E402

d, logp = sys.argv[1], sys.argv[2]
nq = int(sys.argv[3]) if len(sys.argv) > 3 else 3000
o = OracleVacuum(d)
raw = open(d + "/my.doc_length", "rb").read()
N, = struct.unpack("<i", raw[:4])
avg, = struct.unpack("<d", raw[4:12])
c4 = np.frombuffer(raw[12:], dtype=np.uint8).reshape(N, 5)[:, 4].astype(np.int64)
mant, sh = np.arange(256) & 7, (np.arange(256) >> 3) - 1
lens = np.where(sh < 0, mant, (mant | 8) << np.maximum(sh, 0))
norm = 1.2 * (1 - 0.75 + 0.75 * lens / avg)
idf = lambda df: np.log(1 + (N - df + 0.5) / (df + 0.5))  # noqa: E731
tfn = lambda tf, nm: (tf * 2.2) / (tf + nm)  # noqa: E731
K, SEG, WIN = 10, 63, 2048
tot = pr_glob = pr_win = surv = surv_glob = 0
nblk = blk_all = blk_hit = 0
for q in [l.split() for l in open(logp)][:nq]:
    if min(o.df(t) for t in q) < 10000:
        continue
    (da, ta), (db, tb) = [tuple(map(np.array, o.postings(t))) for t in q]
    A, B = ((da, ta), (db, tb)) if len(da) <= len(db) else ((db, tb), (da, ta))
    D, T = A
    O, OT = B
    ia, io = idf(len(D)), idf(len(O))
    wmax = np.zeros((N + WIN - 1) // WIN, dtype=np.int64)
    np.maximum.at(wmax, O // WIN, OT)
    hit = np.isin(D, O, assume_unique=True)
    otf = np.where(hit, OT[np.minimum(np.searchsorted(O, D), len(O) - 1)], 0)
    nm = norm[c4[D]]
    sd = ia * tfn(T, nm)
    sc = np.where(hit, sd + io * tfn(otf, nm), -1.0)
    ub_g = sd + io * tfn(OT.max(), nm)
    ub_w = sd + io * tfn(wmax[D // WIN], nm)
    nb = (len(D) + 127) // 128
    for s0 in range(0, nb, SEG):
        prev = np.sort(sc[:s0 * 128][sc[:s0 * 128] > 0])[::-1]
        floor = prev[K - 1] if len(prev) >= K else 0.0
        run = np.empty(0)
        for b in range(s0, min(nb, s0 + SEG)):
            thr = max(floor, run[K - 1] if len(run) >= K else 0.0)
            sl = slice(b * 128, min(len(D), b * 128 + 128))
            n = sl.stop - sl.start
            tot += n
            pr_glob += int((ub_g[sl] <= thr).sum())
            pr_win += int((ub_w[sl] <= thr).sum())
            surv += int(hit[sl].sum())
            nblk += 1
            blk_all += bool((ub_g[sl] <= thr).all())
            blk_hit += bool(((ub_g[sl] > thr) & hit[sl]).any())
            surv_glob += int((hit[sl] & (ub_g[sl] > thr)).sum())
            v = sc[sl]
            run = np.sort(np.concatenate([run, v[v > 0]]))[::-1][:K]
print(f"high x high driver postings {tot}: ruled out before the probe by the bound with the "
      f"list's max tf {pr_glob / tot:.3f}, with the 2048-doc window's max tf {pr_win / tot:.3f}; "
      f"survivors scored {surv} -> {surv_glob} with the list bound; blocks {nblk}: every posting ruled out "
      f"{blk_all / nblk:.3f}, no survivor left {1 - blk_hit / nblk:.3f}")
