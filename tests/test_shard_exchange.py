"""Doc-range sharding on CPU with gloo (world_size 2): every rank computes the
heap-insertion events of its doc range (pure-Python model of the reference
ranking), packs them into the product's exchange regions (wiser_amd.shard
REGION LAYOUT: per owner the {count, offset} pairs padded to whole events,
then the slot), moves them with the product's exchange_regions (the
all-to-all wsr_shard_step runs with RCCL), and each owner replays the regions
in shard order; the result must equal the single-engine oracle bit for bit.
Also checks that shard events are a superset of the global insertions."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import DATA, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scored_survivors(post, lens, avg, n, terms):
    import heapmodel as hm
    lists = [post[t] for t in terms]
    common = set(lists[0])
    for p in lists[1:]:
        common &= set(p)
    out = []
    for d in sorted(common):
        s = 0.0
        for t in terms:
            s += hm.idf(n, len(post[t])) * hm.tfn(post[t][d], hm.norm(lens[d], avg))
        out.append((s, d))
    return out


def _worker(rank, world, port, index_dir, queries, k, result_q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import heapmodel as hm
    import struct
    from oracle.oracle import OracleVacuum
    from wiser_amd.shard import exchange_regions, region_events, shard_range, index_doc_count
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = OracleVacuum(index_dir)
    raw = open(os.path.join(index_dir, "my.doc_length"), "rb").read()
    n, avg = struct.unpack_from("<id", raw, 0)
    lens = [raw[12 + 5 * i + 4] for i in range(n)]
    post = {}
    for q in queries:
        for t in q:
            if t not in post:
                d, tf = o.postings(t)
                post[t] = dict(zip(d, tf))
    lo, hi = shard_range(index_doc_count(index_dir), rank, world)
    qpr = len(queries) // world
    counts, events, superset_ok = [], [], True
    for q in queries:
        surv = _scored_survivors(post, lens, avg, n, q)
        mine = [x for x in surv if lo <= x[1] < hi]
        _, ins = hm.rank_stream(mine, k)           # shard events
        _, gins = hm.rank_stream(surv, k)          # global insertions
        superset_ok &= set(g for g in gins if lo <= g[1] < hi) <= set(ins)
        counts.append(len(ins))
        events.extend(ins)
    # the product's regions: owner o's queries o*qpr .. o*qpr+qpr-1
    slot = max(1, max(sum(counts[o_ * qpr:(o_ + 1) * qpr]) for o_ in range(world)) + 3)
    rw = 2 * region_events(qpr, slot)            # int64 words per region
    meta_words = 2 * ((qpr + 1) // 2)
    send = torch.full((world * rw,), -7, dtype=torch.int64)
    ev = 0
    for o_ in range(world):
        base = o_ * rw
        meta = torch.zeros(2 * meta_words, dtype=torch.int32)
        off = 0
        for i in range(qpr):
            c = counts[o_ * qpr + i]
            meta[2 * i], meta[2 * i + 1] = c, off
            for j in range(c):
                s_, d_ = events[ev + j]
                send[base + meta_words + 2 * (off + j)] = struct.unpack("<q", struct.pack("<d", s_))[0]
                send[base + meta_words + 2 * (off + j) + 1] = d_
            ev += c
            off += c
        send[base:base + meta_words] = meta.view(torch.int64)
    recv = exchange_regions(send, world)
    res = []
    for qi in range(qpr):
        stream = []
        for g in range(world):
            base = g * rw
            meta = recv[base:base + meta_words].view(torch.int32)
            c, off = int(meta[2 * qi]), int(meta[2 * qi + 1])
            for j in range(c):
                w0 = int(recv[base + meta_words + 2 * (off + j)])
                stream.append((struct.unpack("<d", struct.pack("<q", w0))[0],
                               int(recv[base + meta_words + 2 * (off + j) + 1])))
        top, _ = hm.rank_stream(stream, k)
        res.append([(d, s) for s, d in top])
    result_q.put((rank, res, superset_ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("k", [3, 10])
def test_gloo_two_rank_exchange_is_exact(indexes, k):
    import random
    from oracle.oracle import OracleVacuum
    d = indexes["wiki5"][0]
    o = OracleVacuum(d)
    toks = open(os.path.join(DATA, "all-tokens.txt")).readline().split()
    freq = sorted(toks, key=lambda t: -o.df(t))[:40]
    rng = random.Random(k)
    queries = [rng.sample(freq, 2) for _ in range(30)] + [[t] for t in rng.sample(freq, 10)]
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, d, queries, k, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(world):
        r, res, sup = q.get(timeout=300)
        out[r] = (res, sup)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    qpr = len(queries) // world
    for r in range(world):
        res, sup = out[r]
        assert sup
        for i, got in enumerate(res):
            want, _ = o.search(queries[r * qpr + i], k)
            assert got == want, queries[r * qpr + i]
