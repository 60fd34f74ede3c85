"""Doc-range shards on one GPU: W shard engines in one process run the device
shard-reduce / pack / owner-replay kernels; the all_to_all is done by tensor
slicing (the collective itself is covered by test_shard_exchange.py with gloo).
Results must equal the unsharded engine and the oracle bit for bit."""
import ctypes as C
import os
import random

import pytest

from conftest import DATA

pytestmark = pytest.mark.gpu


def _run_sharded(index_dir, queries, k, world, phrase=False):
    import torch
    import wiser_amd as w
    from wiser_amd import _capi
    from wiser_amd._capi import check, lib
    from wiser_amd.shard import index_doc_count, shard_range
    qpr = len(queries) // world
    queries = queries[:qpr * world]
    n = index_doc_count(index_dir)
    engs, batches, counts, sends, totals = [], [], [], [], []
    for r in range(world):
        e = w.VacuumEngine(index_dir, doc_range=shard_range(n, r, world))
        e.Load()
        arr = (_capi.Query * len(queries))()
        for i, q in enumerate(queries):
            arr[i] = e.resolve(w.SearchQuery(q, n_results=k, is_phrase=phrase))[0]
        b = w.ResidentBatch(e, len(queries), k)
        b.upload(arr)
        check(lib.wsr_batch_run_events(e._h, b._b))
        cnt = torch.empty(len(queries), dtype=torch.int32, device="cuda")
        tot = (C.c_int64 * world)()
        check(lib.wsr_shard_reduce(e._h, b._b, qpr, world, C.c_void_p(cnt.data_ptr()), tot))
        send = torch.empty((max(sum(tot), 1), 2), dtype=torch.int64, device="cuda")
        check(lib.wsr_shard_pack(e._h, b._b, C.c_void_p(send.data_ptr())))
        engs.append(e); batches.append(b); counts.append(cnt); sends.append(send)
        totals.append(list(tot))
    out = []
    for o in range(world):   # owner o receives slice o of every shard's send buffer
        rcounts = torch.stack([counts[g][o * qpr:(o + 1) * qpr] for g in range(world)]).contiguous()
        parts, rbase, acc = [], [], 0
        for g in range(world):
            start = sum(totals[g][:o])
            parts.append(sends[g][start:start + totals[g][o]])
            rbase.append(acc)
            acc += totals[g][o]
        recv = torch.cat(parts + [torch.zeros((1, 2), dtype=torch.int64, device="cuda")]).contiguous()
        e, b = engs[o], batches[o]
        check(lib.wsr_owner_replay(e._h, b._b, o * qpr, qpr, world, C.c_void_p(rcounts.data_ptr()),
                                   C.c_void_p(recv.data_ptr()), (C.c_uint64 * world)(*rbase)))
        hits = (_capi.Hit * (qpr * k))()
        nh = (C.c_int32 * qpr)()
        check(lib.wsr_batch_fetch_range(e._h, b._b, o * qpr, qpr, hits, nh))
        for i in range(qpr):
            out.append([(hits[i * k + j].doc_id, hits[i * k + j].score) for j in range(nh[i])])
    for b in batches:
        b.close()
    for e in engs:
        e.close()
    return queries, out


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
        qs2, got = _run_sharded(d, qs, k, world)
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
    qs2, got = _run_sharded(d, qs, 10, world)
    for q, g in zip(qs2, got):
        assert g == o.search(q, 10)[0], q
