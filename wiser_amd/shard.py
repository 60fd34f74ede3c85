"""Doc-range sharded serving across GPUs (one process per GPU).

Each rank loads the doc-id range [N*r/W, N*(r+1)/W) of the index and runs every
query of a global batch over that range.  The per-query "events" (survivors a
top-k heap started empty would insert, in doc-id order) are reduced per shard
on the device, exchanged with two all_to_all collectives (RCCL over xGMI on
GPUs, gloo on CPU in tests) and replayed by the query's owner rank in shard
order, which reproduces the single-engine result bit for bit.

Queries of a global batch are owned by contiguous slices: owner(q) = q // qpr.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
from typing import List, Sequence, Tuple

from . import _capi
from ._capi import check, lib

EVENT_WORDS = 2  # one 16-byte Event = two int64 words in the exchange tensors


def index_doc_count(index_dir: str) -> int:
    """Number of doc ids covered by my.doc_length (max id + 1 == count for our writer)."""
    with open(os.path.join(index_dir, "my.doc_length"), "rb") as f:
        (n,) = struct.unpack("<i", f.read(4))
    return n


def shard_range(n_docs: int, rank: int, world: int) -> Tuple[int, int]:
    lo = n_docs * rank // world
    hi = n_docs * (rank + 1) // world
    return lo, hi


def exchange(counts, send, owner_totals: Sequence[int], world: int, qpr: int, group=None):
    """Owner-major exchange of shard events.

    counts: int32 tensor [world * qpr] (events of each query in this shard)
    send:   int64 tensor [sum(owner_totals), 2] (events packed owner-major)
    returns (rcounts int32 [world, qpr] shard-major, recv int64 [*, 2], rbase list)
    """
    import torch
    import torch.distributed as dist
    dev = counts.device
    if dist.get_backend(group) == "gloo" and dev.type != "cpu":
        # gloo moves host tensors only (CPU tests, or GPUs sharing one device)
        rc, rv, rb = exchange(counts.cpu(), send.cpu(), owner_totals, world, qpr, group)
        return rc.to(dev), rv.to(dev), rb
    rcounts = torch.empty((world, qpr), dtype=torch.int32, device=dev)
    dist.all_to_all_single(rcounts.view(-1), counts.view(-1), group=group)
    tot = torch.tensor(list(owner_totals), dtype=torch.int64, device=dev)
    rtot = torch.empty_like(tot)
    dist.all_to_all_single(rtot, tot, group=group)
    rsplit = [int(x) for x in rtot.cpu().tolist()]
    recv = torch.empty((max(sum(rsplit), 1), EVENT_WORDS), dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv[:sum(rsplit)], send[:sum(owner_totals)],
                           output_split_sizes=rsplit, input_split_sizes=list(owner_totals),
                           group=group)
    rbase, acc = [], 0
    for x in rsplit:
        rbase.append(acc)
        acc += x
    return rcounts, recv, rbase


class ShardedSearcher:
    """One rank of a doc-range sharded engine (device = local GPU)."""

    def __init__(self, index_dir: str, rank: int, world: int, device: int = 0,
                 threads: int = 0, group=None, positions: bool = True):
        from .engine import VacuumEngine
        self.rank, self.world, self.group = rank, world, group
        self.n_docs = index_doc_count(index_dir)
        self.doc_range = shard_range(self.n_docs, rank, world)
        self.engine = VacuumEngine(index_dir, device=device, threads=threads,
                                   doc_range=self.doc_range if world > 1 else None,
                                   positions=positions)
        self.engine.Load()
        self._batches = {}

    def batch(self, max_queries: int, k: int):
        from .engine import ResidentBatch
        key = (max_queries, k)
        if key not in self._batches:
            self._batches[key] = ResidentBatch(self.engine, max_queries, k)
        return self._batches[key]

    def run(self, b, qpr: int, fetch: bool = True):
        """Run an uploaded global batch (world * qpr queries); returns this
        rank's owned slice [rank*qpr, (rank+1)*qpr) as (hits, n_hits) ctypes
        arrays (None when fetch is False: results stay in HBM)."""
        import torch
        eng = self.engine
        Q = b.nq
        assert Q == qpr * self.world
        check(lib.wsr_batch_run_events(eng._h, b._b))
        dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
            else torch.device("cpu")
        counts = torch.empty(Q, dtype=torch.int32, device=dev)
        totals = (C.c_int64 * self.world)()
        check(lib.wsr_shard_reduce(eng._h, b._b, qpr, self.world, C.c_void_p(counts.data_ptr()),
                                   totals))
        tot = list(totals)
        send = torch.empty((max(sum(tot), 1), EVENT_WORDS), dtype=torch.int64, device=dev)
        check(lib.wsr_shard_pack(eng._h, b._b, C.c_void_p(send.data_ptr())))
        rcounts, recv, rbase = exchange(counts, send, tot, self.world, qpr, self.group)
        torch.cuda.synchronize()
        rb = (C.c_uint64 * self.world)(*rbase)
        q0 = self.rank * qpr
        check(lib.wsr_owner_replay(eng._h, b._b, q0, qpr, self.world,
                                   C.c_void_p(rcounts.data_ptr()), C.c_void_p(recv.data_ptr()), rb))
        if not fetch:
            return None
        hits = (_capi.Hit * (qpr * b.stride))()
        nh = (C.c_int32 * qpr)()
        check(lib.wsr_batch_fetch_range(eng._h, b._b, q0, qpr, hits, nh))
        return hits, nh

    def close(self):
        for b in self._batches.values():
            b.close()
        self._batches.clear()
        self.engine.close()
