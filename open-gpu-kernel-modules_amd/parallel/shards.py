"""Peer-shard weights over xGMI ("peermem-style P2P shards",
FSDP / ZeRO-3-like inference weights).

The reference's closest capabilities are remote mapping and read duplication
(uvm_va_block.c:11660-11664 accessed_by, :5164 read-duplicate): data lives on
one processor and is either mapped from, or copied to, the others. For a model
that does not fit one GPU but fits the node, the MI355X-first layout is:

  * every rank owns 1/W of every layer's flattened weights - a managed buffer
    whose preferred location is that rank's GPU (so the tiering runtime keeps
    it in HBM, and can still demote it to host / CXL under pressure);
  * before layer k runs, its shards are all-gathered over RCCL into a transient
    full-size HBM buffer; the gather for layer k+1 (k+2, ...) is issued on a
    side comm stream while layer k computes (``depth`` buffers in flight);
  * the gathered buffer is viewed as the layer's named tensors.

xGMI sizing (topology.py): a direct all-gather pulls (W-1)/W of the layer over
W-1 links at once - about (layer_bytes / W) / 153 GB/s, e.g. ~0.8 ms for a 1 GB
layer on 8 GPUs - so layers are the natural bucket: each gather is one large
message, never per-tensor.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional, Sequence

import torch
import torch.distributed as dist

from .. import rt
from . import comm


class UnitGather:
    """Per-unit all-gather pipeline of the sharded model (TieredLlama
    ``parallel="shards"``, config 4).

    Every unit (a weight matrix or LM-head part, in its resting format - packed
    or raw) is cut into ``world`` equal byte shards; rank r owns shard r as a
    managed buffer (preferred location: its GPU, or host DRAM when the residency
    plan streams it). ``get(key)`` returns the whole unit, all-gathered over RCCL
    into one of ``depth`` HBM slots; gathers of the units that follow in
    ``order`` are issued ahead on a side stream while the current one is
    consumed (look-ahead = depth - 1). ``done(key)`` marks the slot reusable
    once the kernels already enqueued on the current stream have read it.

    Collectives are issued in the same order on every rank because the issue
    schedule depends only on the sequence of get() calls, never on timing.

    Reference parallel: remote mapping / read duplication of a block resident on
    another processor (uvm_va_block.c:11660-11664, :5164); xGMI sizing in
    SURVEY.md §2.G (a direct all-gather pulls (W-1)/W of a unit over W-1 links).
    """

    def __init__(self, order: Sequence, shard_of, shard_size, world: int, depth: int = 2,
                 device: Optional[torch.device] = None, dev_index: int = 0):
        self.order = list(order)
        self.pos = {k: i for i, k in enumerate(self.order)}
        self.shard_of = shard_of          # key -> ManagedBuffer holding this rank's shard
        self.size_of = shard_size         # key -> shard bytes (the same on every rank)
        self.S = max(shard_size(k) for k in self.order)
        self.world = world
        self.depth = max(1, depth)
        self.device = device or torch.device("cpu")
        self.cuda = self.device.type == "cuda"
        self.dev_index = dev_index
        self.bufs = [torch.empty(self.S * world, dtype=torch.uint8, device=self.device) for _ in range(self.depth)]
        self.stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.slot_free_ev: list = [None] * self.depth
        self.slot_busy = [False] * self.depth
        self.pending: dict = {}   # key -> (slot, ready event); slot -1: the unit's cached copy
        self.next_issue = 0
        self.next_slot = 0
        self.stats = {"gathers": 0, "bytes_in": 0, "cache_hits": 0}
        # Read duplicates of whole units kept in spare HBM (set_cache): gathered
        # once, then served in place - no collective, no slot.
        self.cache_buf: Optional[torch.Tensor] = None
        self.cache_off: dict = {}
        self.cache_filled: set = set()

    def set_cache(self, buf: torch.Tensor, offsets: dict) -> None:
        """Keep the units in ``offsets`` (key -> byte offset into ``buf``, room
        for shard bytes x world each) gathered: the first use all-gathers into
        the cache, later uses read it. The key set must be the same on every
        rank (it decides which collectives are issued)."""
        self.drain()
        self.cache_buf, self.cache_off, self.cache_filled = buf, dict(offsets), set()

    # ---------------------------------------------------------------- internals
    def _free_slot(self) -> Optional[int]:
        for j in range(self.depth):
            s = (self.next_slot + j) % self.depth
            if not self.slot_busy[s]:
                self.next_slot = (s + 1) % self.depth
                return s
        return None

    def _out(self, key, slot: int) -> torch.Tensor:
        if slot < 0:
            off = self.cache_off[key]
            return self.cache_buf[off:off + self.size_of(key) * self.world]
        return self.bufs[slot]

    def _issue(self, key) -> bool:
        S = self.size_of(key)
        if key in self.cache_off:
            slot = -1
            if key in self.cache_filled:  # a resident read duplicate: nothing to move
                self.pending[key] = (-1, None)
                self.stats["cache_hits"] += 1
                return True
            self.cache_filled.add(key)  # (filled by the gather issued below)
        else:
            slot = self._free_slot()
            if slot is None:
                return False
            self.slot_busy[slot] = True
        buf = self.shard_of(key)
        lease = buf.acquire(self.dev_index, rt.READ, 0, S)
        out = self._out(key, slot)[:S * self.world]
        if self.cuda:
            with torch.cuda.stream(self.stream):
                if slot >= 0 and self.slot_free_ev[slot] is not None:
                    self.stream.wait_event(self.slot_free_ev[slot])
                lease.wait(self.stream.cuda_stream)
                shard = lease.tensor((S,), torch.uint8)
                self._gather(out, shard)
                ev = torch.cuda.Event()
                ev.record(self.stream)
                lease.release(self.stream.cuda_stream)
        else:
            lease.wait(0)
            shard = lease.tensor((S,), torch.uint8)
            self._gather(out, shard)
            ev = None
            lease.release(0)
        self.pending[key] = (slot, ev)
        self.stats["gathers"] += 1
        self.stats["bytes_in"] += S * (self.world - 1)
        return True

    def _gather(self, out: torch.Tensor, shard: torch.Tensor) -> None:
        if self.world > 1 or comm.env().forced:
            comm.all_gather_into(out, shard)  # RCCL: the current (side) stream waits, not the host
        else:
            out[:shard.numel()].copy_(shard)

    def _issue_ahead(self, key) -> None:
        """Issue key's gather (if not yet) and the units that follow it in
        ``order``, up to depth - 1 ahead, strictly in order."""
        n = len(self.order)
        if key not in self.pending:
            # Out-of-order use: gathers issued for units that were skipped are dropped.
            for k in list(self.pending):
                self.done(k)
            self.next_issue = self.pos[key]
        i = self.pos[key]
        # (with a cache the look-ahead runs past cached units: the free slots,
        # not the unit count, bound the gathers in flight)
        limit = max(self.depth, n - 1) if self.cache_off else self.depth
        while (self.next_issue - i) % n < limit:
            k = self.order[self.next_issue]
            if k in self.pending or not self._issue(k):
                break
            self.next_issue = (self.next_issue + 1) % n

    # ---------------------------------------------------------------- API
    def get(self, key) -> torch.Tensor:
        self._issue_ahead(key)
        slot, ev = self.pending[key]
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
        return self._out(key, slot)

    def done(self, key) -> None:
        slot, _ = self.pending.pop(key)
        if slot < 0:  # the cached copy is never rewritten
            return
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self.slot_free_ev[slot] = ev
        self.slot_busy[slot] = False

    def drain(self) -> None:
        for k in list(self.pending):
            self.done(k)
