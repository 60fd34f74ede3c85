#!/usr/bin/env python3
"""HBM bytes per rank of a doc-range shard image (wsr_image_size, host only, no
device) for W = 1, 2, 4, 8, with and without positions, largest shard of each
W.  Usage: image_table.py INDEX_DIR [THREADS] > json"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import wiser_amd as w
    from wiser_amd.shard import index_doc_count, shard_range
    d = sys.argv[1]
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    n = index_doc_count(d)
    out = {"index": d, "n_docs": n, "rows": []}
    for positions in (False, True):
        for world in (1, 2, 4, 8):
            t = time.time()
            sizes = [w.image_size(d, doc_range=shard_range(n, r, world) if world > 1 else None,
                                  positions=positions, threads=threads) for r in range(world)]
            big = max(sizes, key=lambda s: s["total_bytes"])
            out["rows"].append({"world": world, "positions": positions, "max_rank_bytes": big["total_bytes"],
                                "max_rank": big, "sum_bytes": sum(s["total_bytes"] for s in sizes),
                                "seconds": round(time.time() - t, 1)})
            print(f"W={world} positions={positions}: {big['total_bytes'] / 1e9:.2f} GB per rank "
                  f"(sum {out['rows'][-1]['sum_bytes'] / 1e9:.2f} GB)", file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
