"""Doc-range sharded serving across GPUs (one process per GPU).

Each rank loads the doc-id range [N*r/W, N*(r+1)/W) of the index and runs every
query of a global batch over that range.  The per-query "events" (survivors a
top-k heap started empty would insert, in doc-id order) are reduced per shard
on the device as each query's last work item finishes and appended to the
owner's region of an exchange buffer; one all-to-all of whole regions moves
them; the owner replays them in shard order, which reproduces the
single-engine result bit for bit.

Queries of a global batch are owned by contiguous slices: owner(q) = q // qpr.
A region (REGION LAYOUT below) holds the owner's {count, offset} pairs padded
to whole 16-byte events, then a slot of `slot` events, so every size is known
before the step runs (no host round trip inside a step).

  * NativeShardedSearcher: wsr_shard_step, one C call per step -- emission on
    the batch's stream, then one ncclAllToAll of the regions over xGMI and the
    owner replay on the engine's communicator stream.  torch is only the
    launcher's rendezvous (gloo, host side).
  * HostExchangeShardedSearcher: the same device halves
    (wsr_shard_step_emit / wsr_shard_step_replay) with the regions moved by the
    caller's torch.distributed group (exchange_regions): the multi-rank
    rehearsal on one GPU, where RCCL refuses two ranks.
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


# REGION LAYOUT (engine.cc step_emit / step_replay): world regions of
# region_events(qpr, slot) 16-byte events each.  Region o of a sender = the
# int32 pairs {count, offset in the slot} of owner o's queries i = 0..qpr-1 (a
# query of count -1 overflowed the slot), padded to whole events, then the
# slot: the events of those queries, each query's run in doc-id order.  After
# the all-to-all, region g of the owner = what shard g sent it.
def region_events(qpr: int, slot: int) -> int:
    """Events (16 bytes each) of one owner's region."""
    return (qpr + 1) // 2 + slot


def exchange_regions(send, world: int, group=None):
    """The step's all-to-all on the caller's group: send = int64 tensor of
    world regions (region o goes to rank o), returns the world regions
    received (region g came from rank g) -- the layout wsr_shard_step's
    ncclAllToAll moves."""
    import torch
    import torch.distributed as dist
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)   # equal splits: region o -> rank o
    return recv


def slot_for_fill(max_fill: int, qpr: int) -> int:
    """Slot size (events per shard -> owner pair) for an observed largest fill:
    twice it, and never under 8 events per owned query."""
    return int(max(2 * max_fill, 8 * qpr, 1024))


class LoopbackGroup:
    """wsr_loopback: the world ranks of a sharded engine in ONE process (one
    NativeShardedSearcher each, loopback=this), their step groups' all-to-all
    done by device copies between the ranks' exchange buffers -- the RCCL
    path's regions, runs, slots and deferred owner replays at world > 1, with
    only the transport replaced (tests, one-GPU rehearsals).  Every rank must
    submit the same step groups in the same order; destroy after closing the
    searchers."""

    def __init__(self, world: int):
        self.world = world
        self._l = C.c_void_p()
        check(lib.wsr_loopback_create(world, C.byref(self._l)))

    def close(self):
        if self._l:
            lib.wsr_loopback_destroy(self._l)
            self._l = None


class NativeShardedSearcher:
    """One rank of a doc-range sharded engine whose whole step runs in C++
    (wsr_shard_step: run with fused emission + one ncclAllToAll + owner replay)."""

    def __init__(self, index_dir: str, rank: int, world: int, share_id, device: int = 0,
                 threads: int = 0, positions: bool = False, loopback=None):
        """share_id(bytes_or_None) -> bytes: the launcher's rendezvous; rank 0
        passes the RCCL id it made, every rank gets rank 0's id back.
        loopback: a LoopbackGroup instead (every rank in this process, the
        all-to-all by device copies: tests and one-GPU rehearsals)."""
        from .engine import VacuumEngine
        self.rank, self.world = rank, world
        self.n_docs = index_doc_count(index_dir)
        self.doc_range = shard_range(self.n_docs, rank, world)
        self.engine = VacuumEngine(index_dir, device=device, threads=threads,
                                   doc_range=self.doc_range if world > 1 else None, positions=positions)
        self.engine.Load()
        c = C.c_void_p()
        if loopback is not None:
            check(lib.wsr_comm_open_loopback(loopback._l, rank, device, C.byref(c)))
        else:
            uid = (C.c_uint8 * 128)()
            if rank == 0:
                check(lib.wsr_comm_unique_id(uid))
            got = share_id(bytes(uid) if rank == 0 else None)
            uid = (C.c_uint8 * 128).from_buffer_copy(got)
            check(lib.wsr_comm_open(uid, world, rank, device, C.byref(c)))
        self._c = c

    def step(self, b, qpr: int, slot: int):
        """Enqueue one step of an uploaded global batch (world * qpr queries);
        results of the owned slice stay in HBM (fetch_owned reads them)."""
        check(lib.wsr_shard_step(self.engine._h, b._b, self._c, qpr, slot))

    def steps(self, bs, qpr: int, slot: int):
        """A step group (wsr_shard_steps): the batches bs, each of world * qpr
        queries, through one all-to-all."""
        arr = (C.c_void_p * len(bs))(*[b._b for b in bs])
        check(lib.wsr_shard_steps(self.engine._h, arr, len(bs), self._c, qpr, slot))

    def flush(self):
        """Enqueue every deferred owner replay (wsr_comm_flush): after it, a
        device synchronize covers all the work of the steps so far."""
        check(lib.wsr_comm_flush(self._c))

    def max_fill(self, b) -> int:
        tot = (C.c_int64 * self.world)()
        check(lib.wsr_shard_fill(self.engine._h, b._b, self.world, tot))
        return max(tot)

    def fetch_owned(self, b, qpr: int):
        """The owned slice's results.  No flush first: the fetch joins the
        batch's own deferred owner replay (x_join enqueues it, under the
        communicator's lock, from whatever thread fetches), and only that one."""
        hits = (_capi.Hit * (qpr * b.stride))()
        nh = (C.c_int32 * qpr)()
        check(lib.wsr_batch_fetch_range(self.engine._h, b._b, self.rank * qpr, qpr, hits, nh))
        return hits, nh

    def sync_all(self):
        """Every step so far finished on the device (both searchers have it)."""
        self.flush()
        check(lib.wsr_sync(self.engine._h))

    def comm_stats(self) -> dict:
        """Step groups, steps, and where the owner replays ran (wsr_comm_stats_get)."""
        st = _capi.CommStats()
        check(lib.wsr_comm_stats_get(self._c, C.byref(st)))
        return {f: getattr(st, f) for f, _ in st._fields_}

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
        self._send = {}       # per batch: its page-locked send regions (pointer, bytes)
        self._pending = None  # the step whose exchange waits for the next step's launch

    def step(self, b, qpr: int, slot: int):
        """Enqueue the batch's emission (the copy of its send regions to
        page-locked memory included), then finish the previous step: wait for
        its copy, exchange, replay.  So one step's host exchange runs while the
        next step's kernels do."""
        W = self.world
        rb = C.c_uint64()
        check(lib.wsr_shard_step_regions(qpr, slot, C.byref(rb)))
        nbytes = W * rb.value
        if self._pending is not None and self._pending[0] is b:
            self.flush()   # (its send buffer is about to be rewritten)
        ptr, have = self._send.get(id(b), (None, 0))
        if have < nbytes:
            lib.wsr_pinned_free(ptr)
            p = C.c_void_p()
            check(lib.wsr_pinned_alloc(nbytes, C.byref(p)))
            ptr = p.value
            self._send[id(b)] = (ptr, nbytes)
        check(lib.wsr_shard_step_emit_async(self.engine._h, b._b, W, qpr, slot, C.c_void_p(ptr)))
        prev, self._pending = self._pending, (b, qpr, slot, ptr, nbytes)
        if prev is not None:
            self._finish(*prev)

    def _finish(self, b, qpr, slot, ptr, nbytes):
        import torch
        check(lib.wsr_batch_stream_sync(self.engine._h, b._b))
        send = torch.frombuffer((C.c_char * nbytes).from_address(ptr), dtype=torch.int64)
        recv = exchange_regions(send, self.world, self.group)
        # deferred: the owner replay rides in the next run's lean kernel (or is
        # enqueued on the batch's stream by its fetch), as the RCCL path defers it
        check(lib.wsr_shard_step_replay_deferred(self.engine._h, b._b, self.rank, self.world, qpr, slot,
                                                 C.c_void_p(recv.data_ptr())))
        self._keep[(id(b), b.nq)] = (b, recv)   # alive until the replay has run

    def flush(self):
        """Finish the step still waiting for its exchange."""
        prev, self._pending = self._pending, None
        if prev is not None:
            self._finish(*prev)

    def steps(self, bs, qpr: int, slot: int):
        for b in bs:   # (one host exchange per batch: the rehearsal has no collective to share)
            self.step(b, qpr, slot)

    def max_fill(self, b) -> int:
        tot = (C.c_int64 * self.world)()
        check(lib.wsr_shard_fill(self.engine._h, b._b, self.world, tot))
        return max(tot)

    def sync_all(self):
        """Every step so far finished on the device (both searchers have it)."""
        self.flush()
        check(lib.wsr_sync(self.engine._h))

    def fetch_owned(self, b, qpr: int):
        self.flush()
        hits = (_capi.Hit * (qpr * b.stride))()
        nh = (C.c_int32 * qpr)()
        check(lib.wsr_batch_fetch_range(self.engine._h, b._b, self.rank * qpr, qpr, hits, nh))
        return hits, nh

    def close(self):
        self.flush()
        self._keep.clear()
        for ptr, _ in self._send.values():
            lib.wsr_pinned_free(ptr)
        self._send.clear()
        self.engine.close()
