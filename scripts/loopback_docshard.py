"""Device cost of the every-query doc-range form on ONE GPU, with the real
step path (wsr_shard_steps, its regions, slots, deferred owner replays) and
the all-to-all by device copies (loopback communicators, wiser_amd.shard.
LoopbackGroup): the same 4096-query global batches run (a) on W shard engines
of the C3 stand-in, every query on every shard, and (b) on one full-index
engine (the replica).  Both on the same device, pipelined as bench.py's loops
are, so time_replica / time_docshard is the share of the device's work the
W-way split adds -- per-query fixed costs (plan, item setup, emission, owner
replay) paid W times -- with no host exchange and no second process.  What
each GPU of a W-GPU node would do in that form is 1/W of (a).  One JSON line
per W.

usage: loopback_docshard.py [W ...]   (default 2 4 8)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    worlds = [int(x) for x in sys.argv[1:]] or [2, 4, 8]
    import bench
    sys.argv = [sys.argv[0], "--no-cpu"]
    a = bench.parse()
    import wiser_amd as w
    from wiser_amd import _capi
    from wiser_amd.shard import LoopbackGroup, NativeShardedSearcher, slot_for_fill
    idx, qlog, _ = bench.ensure_c3(a)
    lines = [l.split() for l in open(qlog).read().splitlines()]
    B, nb, group, passes = 4096, 16, 4, 3   # 4 groups in rotation: the deferred replays
    # (kReplayLag = 2 groups) ride the lean kernels as in bench.py's loop
    chunks = [lines[i * B:(i + 1) * B] for i in range(nb)]

    def qarr(eng, chunk):
        return (_capi.Query * len(chunk))(*[eng.resolve(w.SearchQuery(q, n_results=10))[0] for q in chunk])

    # (b) the replica: one full image, the same batches, pipelined
    eng = w.VacuumEngine(idx, device=0, threads=bench.HOST_THREADS, positions=False)
    eng.Load()
    bs = []
    for c in chunks:
        b = w.ResidentBatch(eng, B, 10)
        b.upload(qarr(eng, c))
        bs.append(b)
    for b in bs:
        b.run()
    w.sync(eng)
    t0 = time.perf_counter()
    for _ in range(passes):
        for b in bs:
            b.run()
    w.sync(eng)
    rep = passes * nb * B / (time.perf_counter() - t0)
    for b in bs:
        b.close()
    eng.close()
    for W in worlds:
        qpr = B // W
        L = LoopbackGroup(W)
        S = [NativeShardedSearcher(idx, r, W, share_id=None, loopback=L, threads=bench.HOST_THREADS)
             for r in range(W)]
        gb = [[None] * nb for _ in range(W)]
        for r, s in enumerate(S):
            for i, c in enumerate(chunks):
                b = w.ResidentBatch(s.engine, qpr * W, 10)
                b.upload(qarr(s.engine, c[:qpr * W]))
                gb[r][i] = b
        # slot from a first pass's fills (twice the largest, as bench.py sizes it)
        for r, s in enumerate(S):
            s.steps(gb[r][:group], qpr, 64 * qpr)
        fill = max(S[r].max_fill(gb[r][i]) for r in range(W) for i in range(group))
        slot = slot_for_fill(fill, qpr)

        def run_groups():
            for _ in range(passes):
                for g0 in range(0, nb, group):
                    for r, s in enumerate(S):
                        s.steps(gb[r][g0:g0 + group], qpr, slot)
            for s in S:
                s.sync_all()
        run_groups()   # warm
        t0 = time.perf_counter()
        run_groups()
        el = time.perf_counter() - t0
        ds = passes * nb * qpr * W / el
        stats = S[0].comm_stats()
        for row in gb:
            for b in row:
                b.close()
        for s in S:
            s.close()
        L.close()
        print(json.dumps({"world": W, "docshard_qps_one_gpu": round(ds, 1), "replica_qps": round(rep, 1),
                          "docshard_over_replica": round(ds / rep, 3), "slot_events": slot,
                          "comm": stats, "batch": B, "q_per_owner": qpr,
                          "note": "every query on W doc-range shards of the C3 stand-in, all on one GPU, "
                                  "loopback all-to-all (device copies); the replica: one full image"}),
              flush=True)


if __name__ == "__main__":
    main()
