#!/usr/bin/env python3
"""How much could block-max pruning skip on the C2 high x high class? (VERDICT
r1 #2; measurement only, CPU, numpy over the oracle's decoded lists.)

For the two-term queries whose lists both have df >= 10k, walk the driver's
128-posting blocks in segments of the lean kernel's length (42 blocks) and
count the blocks whose every score is <= the threshold a segment could know
before the block -- max(k-th best of all earlier segments, the segment's own
running k-th best): no such block can hold a heap insertion.  Then count the
blocks a bound can rule out without probing the other list, using
  exact driver part: max over the block of idf_d * tfn(tf, norm(len)), plus
  other part:        idf_o * tfn(max tf of the other list in the block's doc
                     window (2048-doc windows), norm(shortest doc of the block)).
Usage: blockmax_estimate.py INDEX_DIR LOG [N_QUERIES]"""
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
K, SEG, WIN = 10, 42, 2048
tot = none_ins = bound_ok = 0
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
    nb = (len(D) + 127) // 128
    for s0 in range(0, nb, SEG):
        prev = np.sort(sc[:s0 * 128][sc[:s0 * 128] > 0])[::-1]
        floor = prev[K - 1] if len(prev) >= K else 0.0
        run = []
        for b in range(s0, min(nb, s0 + SEG)):
            tot += 1
            r = sorted(run, reverse=True)
            thr = max(floor, r[K - 1] if len(r) >= K else 0.0)
            sl = slice(b * 128, min(len(D), b * 128 + 128))
            v = sc[sl]
            none_ins += v.max() <= thr
            ub = sd[sl].max() + io * tfn(wmax[D[sl][0] // WIN:D[sl][-1] // WIN + 1].max(), norm[c4[D[sl]].min()])
            bound_ok += ub <= thr
            run.extend(v[v > 0].tolist())
print(f"high x high driver blocks {tot}: no insertion possible in {none_ins / tot:.3f}, "
      f"ruled out by the bound {bound_ok / tot:.3f}")
