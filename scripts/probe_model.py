"""Lines per driver block of the lean kernel's O1 probe under two index
structures (CPU model over a log, diagnostics only).

  bitmap   the rank bitmap (a 4-byte mask word per 32 docs, 1,024 docs per
           128-byte line; a hit's 8-byte rank record, 512 docs per line);
  offsets  per container of w docs (w a power of two, chosen per list so that a
           container holds ~M postings on average) one u32 entry (rank << 8 |
           count) in a rank array, and per posting one byte (its doc's offset
           in its container) in posting order: a probe reads the rank entry of
           its doc's container (a window of the entries the driver block spans
           is loaded coalesced, one entry per lane and dword) and the
           container's offset bytes (one 12-byte load), a hit then its tf byte.

For the first BATCH two-term queries of the log whose other list is long
enough to be probed (df >= span / 2048) it counts, per driver block, the
distinct 128-byte lines each scheme reads (no pruning; the kernel's pre-probe
bound drops some postings of both schemes alike).

usage: probe_model.py INDEX_DIR LOG [BATCH] [M]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LINE = 128


def lines(byte_addrs):
    return len(np.unique(np.asarray(byte_addrs, dtype=np.int64) // LINE)) if len(byte_addrs) else 0


def main():
    from oracle.oracle import OracleVacuum
    idx, log = sys.argv[1], sys.argv[2]
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    mean = float(sys.argv[4]) if len(sys.argv) > 4 else 3.0
    o = OracleVacuum(idx)
    raw = open(os.path.join(idx, "my.doc_length"), "rb").read(4)
    n_docs = int(np.frombuffer(raw, dtype=np.int32)[0])
    dense_df = n_docs // 2048
    cache = {}

    def plist(t):
        if t not in cache:
            d, tf = o.postings(t)
            cache[t] = (np.asarray(d, dtype=np.int64), np.asarray(tf, dtype=np.int64))
        return cache[t]

    qs = [l.split() for l in open(log).read().splitlines()][:batch]
    tot = dict(blocks=0, bm_mask=0, bm_rank=0, off_win=0, off_slow=0, off_low=0, off_tf=0, hits=0,
               win_blocks=0, slow_blocks=0, over=0, probes=0, drv=0, o1_algo=0)
    by_w = {}
    for window in (64, 128):
        pass
    for t in qs:
        if len(t) != 2 or o.df(t[0]) == 0 or o.df(t[1]) == 0:
            continue
        a, b = plist(t[0]), plist(t[1])
        (drv, _), (oth, otf) = (a, b) if len(a[0]) <= len(b[0]) else (b, a)
        if len(oth) < dense_df:
            continue
        p = len(oth) / n_docs
        # container width: a power of two in [16, 256] with ~`mean` postings
        w = int(2 ** np.clip(np.round(np.log2(mean / p)), 4, 8))
        by_w[w] = by_w.get(w, 0) + 1
        cont = oth // w
        ranks = np.searchsorted(cont, np.arange(0, n_docs // w + 2))   # rank at container start
        pos_in_o = {int(d): i for i, d in enumerate(oth.tolist())}
        for s in range(0, len(drv), 128):
            blk = drv[s:s + 128]
            prev = drv[s - 1] + 1 if s else 0
            tot["blocks"] += 1
            tot["probes"] += len(blk)
            hit = np.isin(blk, oth)
            hd = blk[hit]
            tot["hits"] += len(hd)
            # bitmap: mask words (4 B per 32 docs), rank records of hits (8 B per 32 docs)
            tot["bm_mask"] += lines((blk // 32) * 4)
            tot["bm_rank"] += lines((hd // 32) * 8)
            # offsets: the rank entries the block spans, one window load when they fit
            c0, c1 = prev // w, blk[-1] // w
            if c1 - c0 + 2 <= 128:
                tot["win_blocks"] += 1
                tot["off_win"] += lines(np.arange(c0, c1 + 2) * 4)
            else:
                tot["slow_blocks"] += 1
                cb = blk // w
                tot["off_slow"] += lines(np.concatenate([cb * 4, (cb + 1) * 4]))
            cb = blk // w
            r0 = ranks[cb]
            cnt = ranks[cb + 1] - r0
            nz = cnt > 0
            tot["over"] += int(np.sum(cnt > 9))
            tot["off_low"] += lines(np.concatenate([r0[nz], r0[nz] + np.minimum(cnt[nz], 12) - 1]))
            tot["off_tf"] += lines(np.array([pos_in_o[int(d)] for d in hd], dtype=np.int64))
            # O1's compressed postings over the block's doc range (algorithmic bytes)
            lo_i, hi_i = np.searchsorted(oth, [prev, blk[-1] + 1])
            n_o = hi_i - lo_i
            bits = max(1.0, np.log2(max(2.0, (blk[-1] + 1 - prev) / max(1, n_o)))) + 1
            tot["o1_algo"] += n_o * (bits + 2) / 8
    B = max(1, tot["blocks"])
    print(f"{idx}: {B} driver blocks of lean two-term queries (first {batch} of the log); mean "
          f"{mean} postings per container; container widths (queries): {dict(sorted(by_w.items()))}")
    print(f"  probes / block {tot['probes'] / B:.1f}, hits / block {tot['hits'] / B:.2f}")
    bm = (tot["bm_mask"] + tot["bm_rank"]) / B
    print(f"  bitmap : mask lines {tot['bm_mask'] / B:.2f} + rank-record lines {tot['bm_rank'] / B:.2f}"
          f" = {bm:.2f} per block")
    off = (tot["off_win"] + tot["off_slow"] + tot["off_low"] + tot["off_tf"]) / B
    print(f"  offsets: rank window lines {tot['off_win'] / B:.2f} (blocks in one 128-entry window "
          f"{100 * tot['win_blocks'] / B:.1f} %) + per-posting rank lines {tot['off_slow'] / B:.2f} + "
          f"offset-byte lines {tot['off_low'] / B:.2f} + tf lines {tot['off_tf'] / B:.2f} = {off:.2f} per block; "
          f"containers over 9 postings: {tot['over']} of {tot['probes']} probes")
    print(f"  O1 compressed bytes over the blocks' ranges: {tot['o1_algo'] / B / LINE:.2f} lines per block")
    o.close()


if __name__ == "__main__":
    main()
