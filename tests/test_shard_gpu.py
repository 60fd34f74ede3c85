"""Doc-range shards on one GPU: W shard engines in one process run the device
halves of wsr_shard_step (wsr_shard_step_emit: plan + segments with each
query's reduced events emitted into its owner's region; wsr_shard_step_replay:
the owner replay), with the regions moved by copies exactly as the step's
ncclAllToAll moves them (the collective itself is covered by
test_shard_exchange.py with gloo, and with one RCCL rank below).  Results must
equal the oracle bit for bit."""
import ctypes as C
import os
import random

import pytest

from conftest import DATA

pytestmark = pytest.mark.gpu


def open_shards(index_dir, world, positions=False):
    """The W shard engines of a doc-range split of index_dir."""
    import wiser_amd as w
    from wiser_amd.shard import index_doc_count, shard_range
    n = index_doc_count(index_dir)
    engs = []
    try:
        for r in range(world):
            e = w.VacuumEngine(index_dir, doc_range=shard_range(n, r, world), positions=positions)
            e.Load()
            engs.append(e)
    except Exception:
        for e in engs:
            e.close()
        raise
    return engs


def _run_step_regions(index_dir, queries, k, world, slot, phrase=False, engines=None):
    """wsr_shard_step's own buffers at W > 1: every shard runs
    wsr_shard_step_emit (fused emission into the engine's region buffer, owner
    o's {count, offset} block inside region o, region stride = meta + slot), the
    regions are moved exactly as ncclAllToAll moves them (region o of rank g ->
    region g of rank o), and wsr_shard_step_replay replays each owner.  slot
    None: sized from a first emission's fill (wsr_shard_fill), as bench.py does."""
    import numpy as np
    import wiser_amd as w
    from wiser_amd import _capi
    from wiser_amd._capi import check, lib
    from wiser_amd.shard import slot_for_fill
    qpr = len(queries) // world
    queries = queries[:qpr * world]
    engs = engines or open_shards(index_dir, world, positions=phrase)
    batches = []
    try:
        for e in engs:
            arr = (_capi.Query * len(queries))()
            for i, q in enumerate(queries):
                arr[i] = e.resolve(w.SearchQuery(q, n_results=k, is_phrase=phrase))[0]
            b = w.ResidentBatch(e, len(queries), k)
            batches.append(b)
            b.upload(arr)

        def emit(slot):
            rb = C.c_uint64()
            check(lib.wsr_shard_step_regions(qpr, slot, C.byref(rb)))
            words = rb.value // 8
            sends = []
            for e, b in zip(engs, batches):
                send = np.full(world * words, -7, dtype=np.int64)
                check(lib.wsr_shard_step_emit(e._h, b._b, world, qpr, slot, C.c_void_p(send.ctypes.data)))
                sends.append(send.reshape(world, words))
            return sends
        if slot is None:
            sends = emit(64 * qpr)
            fill = 0
            for e, b in zip(engs, batches):
                tot = (C.c_int64 * world)()
                check(lib.wsr_shard_fill(e._h, b._b, world, tot))
                fill = max(fill, max(tot))
            slot = slot_for_fill(fill, qpr)
        sends = emit(slot)
        out = []
        for o in range(world):
            recv = np.ascontiguousarray(np.stack([sends[g][o] for g in range(world)]))
            e, b = engs[o], batches[o]
            check(lib.wsr_shard_step_replay(e._h, b._b, o, world, qpr, slot, C.c_void_p(recv.ctypes.data)))
            hits = (_capi.Hit * (qpr * k))()
            nh = (C.c_int32 * qpr)()
            rc = lib.wsr_batch_fetch_range(e._h, b._b, o * qpr, qpr, hits, nh)
            if rc:
                raise _capi.WiserError(rc, lib.wsr_last_error().decode())
            for i in range(qpr):
                out.append([(hits[i * k + j].doc_id, hits[i * k + j].score) for j in range(nh[i])])
        return queries, out
    finally:
        for b in batches:
            b.close()
        if engines is None:
            for e in engs:
                e.close()


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_sharded_equals_oracle_wiki5(indexes, world):
    from oracle.oracle import OracleVacuum
    d = indexes["wiki5"][0]
    o = OracleVacuum(d)
    toks = open(os.path.join(DATA, "all-tokens.txt")).readline().split()
    freq = sorted(toks, key=lambda t: -o.df(t))[:60]
    rng = random.Random(world)
    qs = ([rng.sample(freq, 2) for _ in range(120)] + [[t] for t in rng.sample(toks, 60)] +
          [rng.sample(toks, 2) for _ in range(60)] + [rng.sample(freq, 3) for _ in range(40)])
    for k in (1, 10):
        qs2, got = _run_step_regions(d, qs, k, world, slot=None)
        for q, g in zip(qs2, got):
            assert g == o.search(q, k)[0], (world, k, q)


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_equals_oracle_synthetic(synth_small, world):
    from oracle.oracle import OracleVacuum
    import wiser_amd as w
    d, _ = synth_small
    log = os.path.join(d, "qshard.log")
    w.gen_two_term_log(d, log, n_queries=800, seed=11)
    qs = [l.split() for l in open(log).read().splitlines()]
    o = OracleVacuum(d)
    qs2, got = _run_step_regions(d, qs, 10, world, slot=None)
    for q, g in zip(qs2, got):
        assert g == o.search(q, 10)[0], q


def test_native_rccl_step_one_rank(synth_small):
    """wsr_shard_step (fused emission, RCCL communicator, one ncclAllToAll,
    owner replay on the communicator's stream) with a communicator of one rank,
    several steps in flight on two batches: equal to the oracle."""
    import wiser_amd as w
    from wiser_amd import _capi
    from wiser_amd.shard import NativeShardedSearcher
    from oracle.oracle import OracleVacuum
    d, _ = synth_small
    log = os.path.join(d, "qshard_native.log")
    w.gen_two_term_log(d, log, n_queries=512, seed=13)
    qs = [l.split() for l in open(log).read().splitlines()]
    S = NativeShardedSearcher(d, 0, 1, share_id=lambda x: x)
    eng = S.engine
    arr = (_capi.Query * len(qs))()
    for i, q in enumerate(qs):
        arr[i] = eng.resolve(w.SearchQuery(q, n_results=10))[0]
    half = len(qs) // 2
    parts = [qs[:half], qs[half:2 * half]]
    bs = []
    for p, part in enumerate(parts):
        b = w.ResidentBatch(eng, half, 10)
        b.upload((_capi.Query * half)(*arr[p * half:(p + 1) * half]))
        bs.append(b)
    for _ in range(3):   # consecutive steps of two batches in flight
        for b in bs:
            S.step(b, half, 64 * half)
    o = OracleVacuum(d)
    for b, part in zip(bs, parts):
        hits, nh = S.fetch_owned(b, half)
        assert S.max_fill(b) > 0
        for i, q in enumerate(part):
            assert [(hits[i * 10 + j].doc_id, hits[i * 10 + j].score) for j in range(nh[i])] == o.search(q, 10)[0], q
    # an overflowing slot fails the fetch loudly
    S.step(bs[0], half, 2)
    with pytest.raises(_capi.WiserError, match="exchange slot"):
        S.fetch_owned(bs[0], half)
    for b in bs:
        b.close()
    S.close()


def test_native_rccl_step_groups(synth_small):
    """wsr_shard_steps: groups of batches through one ncclAllToAll (regions
    of every batch in the first one's buffers), groups of changing size and
    leader in flight one after another: equal to the oracle."""
    import wiser_amd as w
    from wiser_amd import _capi
    from wiser_amd.shard import NativeShardedSearcher
    from oracle.oracle import OracleVacuum
    d, _ = synth_small
    log = os.path.join(d, "qshard_groups.log")
    w.gen_two_term_log(d, log, n_queries=1024, seed=17)
    qs = [l.split() for l in open(log).read().splitlines()]
    S = NativeShardedSearcher(d, 0, 1, share_id=lambda x: x)
    eng = S.engine
    n = 256
    parts = [qs[i * n:(i + 1) * n] for i in range(4)]
    bs = []
    for part in parts:
        arr = (_capi.Query * n)(*[eng.resolve(w.SearchQuery(q, n_results=10))[0] for q in part])
        b = w.ResidentBatch(eng, n, 10)
        b.upload(arr)
        bs.append(b)
    o = OracleVacuum(d)
    exp = [[o.search(q, 10)[0] for q in part] for part in parts]
    for order in ([0, 1, 2], [3], [1, 3, 0, 2], [2, 0], [0, 1, 2, 3]):
        S.steps([bs[i] for i in order], n, 64 * n)
    for b, e in zip(bs, exp):
        hits, nh = S.fetch_owned(b, n)
        got = [[(hits[i * 10 + j].doc_id, hits[i * 10 + j].score) for j in range(nh[i])] for i in range(n)]
        assert got == e
    for b in bs:
        b.close()
    S.close()


@pytest.mark.parametrize("defer", ["1", "0"])
def test_native_rccl_deferred_replay(synth_small, monkeypatch, defer):
    """Owner replays deferred into later groups' lean kernels (the default)
    and not (WSR_REPLAY_DEFER=0): 14 step groups of changing size over five
    batches -- one of k = 100, whose replay needs the LDS heap and so is never
    deferred -- more groups than exchange buffer sets, batches stepped again
    while their replay is pending; then a flush and every fetch, and again
    with fetches straight after the steps.  Each phase runs a query set the
    batches did not hold before, so a replay left undone shows.  Equal to the
    oracle."""
    import wiser_amd as w
    from wiser_amd import _capi
    from wiser_amd.shard import NativeShardedSearcher, slot_for_fill
    from oracle.oracle import OracleVacuum
    monkeypatch.setenv("WSR_REPLAY_DEFER", defer)
    d, _ = synth_small
    log = os.path.join(d, "qshard_defer.log")
    w.gen_two_term_log(d, log, n_queries=3 * 1280, seed=23)
    qs = [l.split() for l in open(log).read().splitlines()]
    S = NativeShardedSearcher(d, 0, 1, share_id=lambda x: x)
    eng = S.engine
    n = 256
    ks = [10, 10, 10, 10, 100]
    o = OracleVacuum(d)
    sets = [[qs[(5 * s + i) * n:(5 * s + i + 1) * n] for i in range(5)] for s in range(3)]
    bs = [w.ResidentBatch(eng, n, k) for k in ks]

    def upload(parts):
        for b, part, k in zip(bs, parts, ks):
            b.upload((_capi.Query * n)(*[eng.resolve(w.SearchQuery(q, n_results=k))[0] for q in part]))
        return [[o.search(q, k)[0] for q in part] for part, k in zip(parts, ks)]

    def check(exp):
        for b, e in zip(bs, exp):
            hits, nh = S.fetch_owned(b, n)
            got = [[(hits[i * b.stride + j].doc_id, hits[i * b.stride + j].score) for j in range(nh[i])]
                   for i in range(n)]
            assert got == e

    groups = [[0, 1], [2, 3], [4], [0, 1, 2], [3, 4], [1], [2, 0], [4, 3, 1], [0], [1, 2, 3, 4], [0, 4], [2],
              [3], [1, 0]]
    try:
        # the slot from a first pass (the k = 100 batch sends every survivor)
        upload(sets[0])
        for b in bs:
            S.steps([b], n, 1 << 20)
        slot = slot_for_fill(max(S.max_fill(b) for b in bs), n)
        exp = upload(sets[1])
        for g in groups:
            S.steps([bs[i] for i in g], n, slot)
        S.flush()
        w.sync(eng)
        check(exp)
        exp = upload(sets[2])
        for g in groups[:5]:
            S.steps([bs[i] for i in g], n, slot)
        check(exp)
    finally:
        for b in bs:
            b.close()
        S.close()


def test_native_rccl_failed_group_flushes_predecessor(synth_small, monkeypatch):
    """a step group whose emission fails after it has taken the
    deferred replays of an earlier group must still enqueue them: the earlier
    group's batches are then fetched (bit-exact) and destroyed without waiting
    forever in x_join.  The failure is injected (wsr_debug_fail_runs)."""
    import wiser_amd as w
    from wiser_amd import _capi
    from wiser_amd._capi import lib
    from wiser_amd.shard import NativeShardedSearcher, slot_for_fill
    from oracle.oracle import OracleVacuum
    monkeypatch.setenv("WSR_REPLAY_DEFER", "1")
    d, _ = synth_small
    log = os.path.join(d, "qshard_fail.log")
    w.gen_two_term_log(d, log, n_queries=4 * 256, seed=29)
    qs = [l.split() for l in open(log).read().splitlines()]
    S = NativeShardedSearcher(d, 0, 1, share_id=lambda x: x)
    eng = S.engine
    n = 256
    o = OracleVacuum(d)
    bs = [w.ResidentBatch(eng, n, 10) for _ in range(3)]
    try:
        parts = [qs[i * n:(i + 1) * n] for i in range(3)]
        for b, part in zip(bs, parts):
            b.upload((_capi.Query * n)(*[eng.resolve(w.SearchQuery(q, n_results=10))[0] for q in part]))
        S.steps([bs[0]], n, 1 << 20)
        slot = slot_for_fill(S.max_fill(bs[0]), n)
        S.steps([bs[0]], n, slot)   # group 0
        S.steps([bs[1]], n, slot)   # group 1
        lib.wsr_debug_fail_runs(1)
        try:
            with pytest.raises(RuntimeError):
                S.steps([bs[2]], n, slot)   # takes group 0's replays, then fails
        finally:
            lib.wsr_debug_fail_runs(0)
        for i in (0, 1):
            hits, nh = S.fetch_owned(bs[i], n)
            got = [[(hits[q * 10 + j].doc_id, hits[q * 10 + j].score) for j in range(nh[q])] for q in range(n)]
            assert got == [o.search(q, 10)[0] for q in parts[i]]
    finally:
        for b in bs:
            b.close()
        S.close()


def test_host_exchange_pipelined(synth_small):
    """HostExchangeShardedSearcher (the gloo rehearsal's searcher): each step
    enqueues its emission and then finishes the step before it (exchange,
    replay), the same batch twice in a row included; a one-rank gloo group in
    this process.  Equal to the oracle."""
    import torch.distributed as dist
    import wiser_amd as w
    from wiser_amd import _capi
    from wiser_amd.shard import HostExchangeShardedSearcher
    from oracle.oracle import OracleVacuum
    d, _ = synth_small
    log = os.path.join(d, "qshard_hostx.log")
    w.gen_two_term_log(d, log, n_queries=1024, seed=19)
    qs = [l.split() for l in open(log).read().splitlines()]
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:29613", rank=0, world_size=1)
    try:
        S = HostExchangeShardedSearcher(d, 0, 1)
        eng = S.engine
        n = 256
        parts = [qs[i * n:(i + 1) * n] for i in range(4)]
        bs = []
        for part in parts:
            arr = (_capi.Query * n)(*[eng.resolve(w.SearchQuery(q, n_results=10))[0] for q in part])
            b = w.ResidentBatch(eng, n, 10)
            b.upload(arr)
            bs.append(b)
        for i in (0, 1, 2, 3, 3, 1, 0, 2):
            S.step(bs[i], n, 64 * n)
        o = OracleVacuum(d)
        for b, part in zip(bs, parts):
            hits, nh = S.fetch_owned(b, n)
            got = [[(hits[i * 10 + j].doc_id, hits[i * 10 + j].score) for j in range(nh[i])] for i in range(n)]
            assert got == [o.search(q, 10)[0] for q in part]
        for b in bs:
            b.close()
        S.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,k", [(2, 10), (3, 10), (8, 10), (3, 200)])
def test_step_regions_equal_oracle(synth_small, world, k):
    """The native step's region layout (in-region meta, region stride, one
    all-to-all of whole regions) at W = 2, 3, 8, narrow and wide k."""
    from oracle.oracle import OracleVacuum
    import wiser_amd as w
    d, _ = synth_small
    log = os.path.join(d, "qshard_regions.log")
    w.gen_two_term_log(d, log, n_queries=960, seed=17)
    qs = [l.split() for l in open(log).read().splitlines()]
    if k > 64:
        qs = qs[:240]
    o = OracleVacuum(d)
    qpr = len(qs) // world
    # an odd q_per_owner pads the meta block to whole events
    if qpr % 2 == 0:
        qpr -= 1
    qs = qs[:qpr * world]
    qs2, got = _run_step_regions(d, qs, k, world, slot=(4096 if k > 64 else 64) * qpr)
    for q, g in zip(qs2, got):
        assert g == o.search(q, k)[0], (world, k, q)


def test_step_regions_overflow_is_loud(synth_small):
    import wiser_amd as w  # noqa: F401
    from wiser_amd import _capi
    d, _ = synth_small
    head = [f"t{i:07d}" for i in range(8)]
    qs = [[head[i % 8], head[(i + 1) % 8]] for i in range(64)]
    with pytest.raises(_capi.WiserError, match="exchange slot"):
        _run_step_regions(d, qs, 10, 2, slot=4)


def test_host_replay_taken_by_phrase_only_run(positions_index):
    """a deferred host-exchange owner replay taken by a plain
    run of a phrase-only batch (no conjunctive lean item) must still run -- the
    conjunctive launch that carries it is forced -- and the owner's fetch must
    wait for it.  Both batches equal the oracle."""
    import torch.distributed as dist
    import wiser_amd as w
    from wiser_amd import _capi
    from wiser_amd.shard import HostExchangeShardedSearcher
    from oracle.oracle import OracleVacuum
    from conftest import phrase_cases
    d, seqs = positions_index
    rng = random.Random(23)
    words = [f"w{i}" for i in range(60)]
    conj = [rng.sample(words[:30], 2) for _ in range(128)]
    phr = [p for p in phrase_cases(seqs, 400, seed=29) if len(p) == 2][:96]
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:29617", rank=0, world_size=1)
    try:
        S = HostExchangeShardedSearcher(d, 0, 1, positions=True)
        eng = S.engine
        o = OracleVacuum(d)
        ba = w.ResidentBatch(eng, len(conj), 10)
        ba.upload((_capi.Query * len(conj))(*[eng.resolve(w.SearchQuery(q, n_results=10))[0] for q in conj]))
        bp = w.ResidentBatch(eng, len(phr), 10)
        bp.upload((_capi.Query * len(phr))(
            *[eng.resolve(w.SearchQuery(q, n_results=10, is_phrase=True))[0] for q in phr]))
        for _ in range(2):
            S.step(ba, len(conj), 64 * len(conj))
            S.flush()          # ba's owner replay now waits for another batch's run
            bp.run()           # a phrase-only run takes it
            hits, nh = bp.fetch()
            for i, q in enumerate(phr):
                got = [(hits[i * 10 + j].doc_id, hits[i * 10 + j].score) for j in range(nh[i])]
                assert got == o.search(q, 10, phrase=True)[0], q
            hits, nh = S.fetch_owned(ba, len(conj))
            got = [[(hits[i * 10 + j].doc_id, hits[i * 10 + j].score) for j in range(nh[i])]
                   for i in range(len(conj))]
            assert got == [o.search(q, 10)[0] for q in conj]
        ba.close()
        bp.close()
        S.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,defer", [(2, "1"), (3, "1"), (3, "0"), (8, "1")])
def test_loopback_shard_steps(synth_small, monkeypatch, world, defer):
    """wsr_shard_steps itself at world > 1 (the W > 1 parity tests
    moved regions by copies outside the step): W doc-range shard engines in
    this process, each with a loopback communicator, so the step groups'
    regions, runs of regions, slots and deferred owner replays run exactly as
    over RCCL, with the all-to-all done by device copies.  Groups of changing
    size and order, more groups than exchange buffer sets, a batch stepped
    again while its replay is pending; every rank's owned slice equal to the
    oracle."""
    import wiser_amd as w
    from wiser_amd import _capi
    from wiser_amd.shard import LoopbackGroup, NativeShardedSearcher
    from oracle.oracle import OracleVacuum
    monkeypatch.setenv("WSR_REPLAY_DEFER", defer)
    d, _ = synth_small
    log = os.path.join(d, f"qshard_loop{world}.log")
    qpr = 96
    nb = 4
    w.gen_two_term_log(d, log, n_queries=nb * world * qpr, seed=29 + world)
    qs = [l.split() for l in open(log).read().splitlines()]
    parts = [qs[i * world * qpr:(i + 1) * world * qpr] for i in range(nb)]
    o = OracleVacuum(d)
    exp = [[o.search(q, 10)[0] for q in part] for part in parts]
    L = LoopbackGroup(world)
    S = [NativeShardedSearcher(d, r, world, share_id=None, loopback=L) for r in range(world)]
    bs = []
    try:
        for s in S:
            row = []
            for part in parts:
                b = w.ResidentBatch(s.engine, world * qpr, 10)
                b.upload((_capi.Query * len(part))(
                    *[s.engine.resolve(w.SearchQuery(q, n_results=10))[0] for q in part]))
                row.append(b)
            bs.append(row)
        slot = 64 * qpr
        for order in ([0, 1], [2], [3, 0], [1, 2, 3], [0], [2, 1], [3]):
            for r, s in enumerate(S):   # every rank submits the group before the next group
                s.steps([bs[r][i] for i in order], qpr, slot)
        for r, s in enumerate(S):
            for i in range(nb):
                hits, nh = s.fetch_owned(bs[r][i], qpr)
                got = [[(hits[q * 10 + j].doc_id, hits[q * 10 + j].score) for j in range(nh[q])]
                       for q in range(qpr)]
                assert got == exp[i][r * qpr:(r + 1) * qpr], (world, r, i)
        st = S[0].comm_stats()
        assert st["groups"] == 7 and st["steps"] == 12
    finally:
        for row in bs:
            for b in row:
                b.close()
        for s in S:
            s.close()
        L.close()
