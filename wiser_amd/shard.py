"""Doc-range sharded serving across GPUs (one process per GPU).

Each rank loads the doc-id range [N*r/W, N*(r+1)/W) of the index and runs every
query of a global batch over that range.  The per-query "events" (survivors a
top-k heap started empty would insert, in doc-id order) are reduced per shard
on the device, exchanged with two all_to_all collectives (RCCL over xGMI on
GPUs, gloo on CPU in tests) and replayed by the query's owner rank in shard
order, which reproduces the single-engine result bit for bit.

Queries of a global batch are owned by contiguous slices: owner(q) = q // qpr.

Two exchanges, both with every size known before the step runs (no host
round trip inside a step):
  * NativeShardedSearcher: wsr_shard_step, one C call per step -- the engine
    packs each owner's events into a fixed slot, RCCL moves counts and slots
    with grouped send / recv over xGMI, the owner replays; all on the batch's
    HIP stream.  torch is only the launcher's rendezvous (gloo, host side).
  * HostExchangeShardedSearcher: the same fused device halves with the
    transfer done by torch.distributed (gloo): the multi-rank rehearsal on one
    GPU, where RCCL refuses two ranks;
  * ShardedSearcher: the earlier split form (reduce, pack, replay launches)
    exchanged by torch.distributed all_to_all (gloo on the CPU in tests).
A slot that overflows fails the batch loudly (error flag at fetch); the slot
size comes from the measured fill (slot_for_fill).
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


def exchange_fixed(counts, send, world: int, qpr: int, slot: int, group=None, out=None):
    """Fixed-slot exchange: counts int32 [world * qpr] (query order), send
    int64 [world * slot, 2] (owner-major slots) -> (rcounts int32 [world, qpr]
    shard-major, recv int64 [world * slot, 2] shard-major), into `out` when
    given.  Equal splits, so no size is read back."""
    import torch
    import torch.distributed as dist
    dev = counts.device
    if out is None:
        out = (torch.empty((world, qpr), dtype=torch.int32, device=dev),
               torch.empty((world * slot, EVENT_WORDS), dtype=torch.int64, device=dev))
    rcounts, recv = out
    if dist.get_backend(group) == "gloo" and dev.type != "cpu":
        rc, rv = exchange_fixed(counts.cpu(), send.cpu(), world, qpr, slot, group)
        rcounts.copy_(rc)
        recv.copy_(rv)
        return rcounts, recv
    dist.all_to_all_single(rcounts.view(-1), counts.view(-1), group=group)
    dist.all_to_all_single(recv, send, group=group)
    return rcounts, recv


def slot_for_fill(max_fill: int, qpr: int) -> int:
    """Slot size (events per shard -> owner pair) for an observed largest fill:
    twice it, and never under 8 events per owned query."""
    return int(max(2 * max_fill, 8 * qpr, 1024))


class NativeShardedSearcher:
    """One rank of a doc-range sharded engine whose whole step runs in C++
    (wsr_shard_step: run with fused emission + one ncclAllToAll + owner replay)."""

    def __init__(self, index_dir: str, rank: int, world: int, share_id, device: int = 0,
                 threads: int = 0, positions: bool = False):
        """share_id(bytes_or_None) -> bytes: the launcher's rendezvous; rank 0
        passes the RCCL id it made, every rank gets rank 0's id back."""
        from .engine import VacuumEngine
        self.rank, self.world = rank, world
        self.n_docs = index_doc_count(index_dir)
        self.doc_range = shard_range(self.n_docs, rank, world)
        self.engine = VacuumEngine(index_dir, device=device, threads=threads,
                                   doc_range=self.doc_range if world > 1 else None, positions=positions)
        self.engine.Load()
        uid = (C.c_uint8 * 128)()
        if rank == 0:
            check(lib.wsr_comm_unique_id(uid))
        got = share_id(bytes(uid) if rank == 0 else None)
        uid = (C.c_uint8 * 128).from_buffer_copy(got)
        c = C.c_void_p()
        check(lib.wsr_comm_open(uid, world, rank, device, C.byref(c)))
        self._c = c

    def step(self, b, qpr: int, slot: int):
        """Enqueue one step of an uploaded global batch (world * qpr queries);
        results of the owned slice stay in HBM (fetch_owned reads them)."""
        check(lib.wsr_shard_step(self.engine._h, b._b, self._c, qpr, slot))

    def max_fill(self, b) -> int:
        tot = (C.c_int64 * self.world)()
        check(lib.wsr_shard_fill(self.engine._h, b._b, self.world, tot))
        return max(tot)

    def fetch_owned(self, b, qpr: int):
        hits = (_capi.Hit * (qpr * b.stride))()
        nh = (C.c_int32 * qpr)()
        check(lib.wsr_batch_fetch_range(self.engine._h, b._b, self.rank * qpr, qpr, hits, nh))
        return hits, nh

    def close(self):
        if self._c:
            lib.wsr_comm_close(self._c)
            self._c = None
        self.engine.close()


class HostExchangeShardedSearcher:
    """The step of NativeShardedSearcher with the transfer done by the caller's
    torch.distributed group instead of RCCL, over the same buffers:
    wsr_shard_step_emit (the segments append each query's reduced events to its
    owner's region of the engine's send buffer, which is copied to the host),
    one all_to_all of whole regions -- the exact layout wsr_shard_step's
    ncclAllToAll moves -- and wsr_shard_step_replay.  This is the multi-rank
    rehearsal on ONE GPU (RCCL refuses two ranks on one device): the gloo group
    moves host copies, so it checks the orchestration, the region layout and the
    results, not the exchange's speed.  Same step / max_fill / fetch_owned / close."""

    def __init__(self, index_dir: str, rank: int, world: int, group=None, device: int = 0,
                 threads: int = 0, positions: bool = False):
        from .engine import VacuumEngine
        self.rank, self.world, self.group = rank, world, group
        self.n_docs = index_doc_count(index_dir)
        self.doc_range = shard_range(self.n_docs, rank, world)
        self.engine = VacuumEngine(index_dir, device=device, threads=threads,
                                   doc_range=self.doc_range if world > 1 else None, positions=positions)
        self.engine.Load()
        self._keep = {}

    def step(self, b, qpr: int, slot: int):
        import torch
        import torch.distributed as dist
        W = self.world
        rb = C.c_uint64()
        check(lib.wsr_shard_step_regions(qpr, slot, C.byref(rb)))
        send = torch.empty(W * rb.value // 8, dtype=torch.int64)
        check(lib.wsr_shard_step_emit(self.engine._h, b._b, W, qpr, slot, C.c_void_p(send.data_ptr())))
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)   # region o -> rank o, equal splits
        check(lib.wsr_shard_step_replay(self.engine._h, b._b, self.rank, W, qpr, slot,
                                        C.c_void_p(recv.data_ptr())))
        self._keep[(id(b), b.nq)] = (b, send, recv)   # alive until the replay has run

    def max_fill(self, b) -> int:
        tot = (C.c_int64 * self.world)()
        check(lib.wsr_shard_fill(self.engine._h, b._b, self.world, tot))
        return max(tot)

    def fetch_owned(self, b, qpr: int):
        hits = (_capi.Hit * (qpr * b.stride))()
        nh = (C.c_int32 * qpr)()
        check(lib.wsr_batch_fetch_range(self.engine._h, b._b, self.rank * qpr, qpr, hits, nh))
        return hits, nh

    def close(self):
        self._keep.clear()
        self.engine.close()


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
        self._xbufs = {}

    def batch(self, max_queries: int, k: int):
        from .engine import ResidentBatch
        key = (max_queries, k)
        if key not in self._batches:
            self._batches[key] = ResidentBatch(self.engine, max_queries, k)
        return self._batches[key]

    def run(self, b, qpr: int, fetch: bool = True, slot: int = 0):
        """Run an uploaded global batch (world * qpr queries); returns this
        rank's owned slice [rank*qpr, (rank+1)*qpr) as (hits, n_hits) ctypes
        arrays (None when fetch is False: results stay in HBM).  The fixed-slot
        exchange (slot events per pair; 0 = 32 per owned query) is ordered on
        the batch's stream, so nothing waits on the host inside the step."""
        import torch
        eng = self.engine
        Q = b.nq
        assert Q == qpr * self.world
        slot = slot or 32 * qpr
        check(lib.wsr_batch_run_events(eng._h, b._b))
        on_gpu = torch.cuda.is_available()
        dev = torch.device("cuda", eng.device) if on_gpu else torch.device("cpu")
        # per batch and slot size: buffers used only in the batch's stream order
        key = (id(b), slot, Q, self.world)
        if key not in self._xbufs:
            self._xbufs[key] = (b,) + (
                torch.empty(Q, dtype=torch.int32, device=dev),
                torch.empty((self.world * slot, EVENT_WORDS), dtype=torch.int64, device=dev),
                torch.empty((self.world, qpr), dtype=torch.int32, device=dev),
                torch.empty((self.world * slot, EVENT_WORDS), dtype=torch.int64, device=dev))
        _, counts, send, rc_buf, rv_buf = self._xbufs[key]
        assert counts.numel() >= b.nq
        check(lib.wsr_shard_pack_fixed(eng._h, b._b, qpr, self.world, slot, C.c_void_p(counts.data_ptr()),
                                       C.c_void_p(send.data_ptr())))
        st = C.c_void_p()
        check(lib.wsr_batch_stream(eng._h, b._b, C.byref(st)))
        if on_gpu:   # the collectives go on the batch's stream, after the pack
            with torch.cuda.stream(torch.cuda.ExternalStream(st.value, device=dev)):
                rcounts, recv = exchange_fixed(counts, send, self.world, qpr, slot, self.group,
                                               out=(rc_buf, rv_buf))
        else:
            rcounts, recv = exchange_fixed(counts, send, self.world, qpr, slot, self.group,
                                           out=(rc_buf, rv_buf))
        q0 = self.rank * qpr
        check(lib.wsr_owner_replay_fixed(eng._h, b._b, q0, qpr, self.world, slot,
                                         C.c_void_p(rcounts.data_ptr()), C.c_void_p(recv.data_ptr())))
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
        self._xbufs.clear()
        self.engine.close()
