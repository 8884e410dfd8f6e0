"""Transparent managed memory for unmodified PyTorch code.

``with ogkm.managed(): model(x)`` runs ordinary torch code on tensors that
oversubscribe HBM. Every aten op is intercepted by a ``TorchDispatchMode``
(the software analog of a GPU page fault, at tensor granularity): before the
op is enqueued, each managed storage it reads or writes takes an *op hold* -
the runtime makes it resident at its stable device VA (evicting cold tensors
to host DRAM through the HBM arena's LRU), pins it, and orders the current
stream after the copies (GPU-side, no host stall). After the op is enqueued
the holds are dropped again: the tensors are evictable, fenced on the stream's
queued uses. A managed tensor's own allocation hold is dropped at its first
use as an operand, so from then on only op holds keep it resident; a tensor
never passed to an op (a library workspace used behind the dispatcher's back)
keeps its allocation hold and is never evicted. Nothing inside the model
calls the framework; tensors the model allocates before the mode is entered
must fit the arena until their first use inside it.

Reference parity: the replayable fault path (fault -> batch service ->
replay, ``uvm_gpu_replayable_faults.c:2906``), the CPU fault entry
(``uvm.c:576``) and prefetch (``uvm_migrate.c:882``); here the operands are
declared by the dispatcher instead of reported by the MMU (no XNACK on this
stack: SURVEY.md §7.1 design (1)).

Layer-ahead prefetch (the D26 prefetcher at op granularity): the mode records
the sequence of managed operand sets of the first pass; on later passes it
recognises its position and prefetches the operands of the next ops (up to
``lookahead_bytes``) right after enqueueing the current one, so the H2D copies
overlap compute.

Tensors become managed when the pluggable allocator is enabled in managed
mode (``allocator.enable(managed_min_mb=N)``, before the first CUDA
allocation): allocations of at least N MB are stable-VA managed ranges.
"""
from __future__ import annotations

from typing import Optional

from ._native import lib

_MODE_CLS = None


def _mode_class():
    global _MODE_CLS
    if _MODE_CLS is not None:
        return _MODE_CLS
    import torch
    from torch.utils._python_dispatch import TorchDispatchMode
    from torch.utils._pytree import tree_flatten

    def _writes_of(func) -> tuple[frozenset, frozenset]:
        """(positional indices, kwarg names) of the arguments the op writes."""
        pos, names = set(), set()
        for i, a in enumerate(func._schema.arguments):
            if a.alias_info is not None and a.alias_info.is_write:
                pos.add(i)
                names.add(a.name)
        return frozenset(pos), frozenset(names)

    class ManagedMode(TorchDispatchMode):
        def __init__(self, device: int = 0, lookahead_bytes: Optional[int] = None):
            super().__init__()
            self.device = int(device)
            # default: a short window - min(512 MB, arena / 16). Measured on the
            # stock 8B model at 2x (12.3 GB arena): 512 MB -> 134 tok/s, 256 MB
            # 125, 0 (no prefetch) 117, 1 GB 62, 2 GB 6.7, a quarter of the arena
            # 4.8: every prefetched tensor is LRU-fresh, so a long window evicts
            # operands needed before the prefetched ones and the passes thrash
            # (profiles/r3_managed_lookahead.txt).
            if lookahead_bytes is None:
                lookahead_bytes = min(512 << 20, _arena_capacity(self.device) // 16)
            self.lookahead_bytes = int(lookahead_bytes)
            self._writes: dict = {}
            self._sizes: dict[int, int] = {}
            self._trace: list[tuple[int, ...]] = []   # operand sets of the recorded pass
            self._first: dict[tuple[int, ...], int] = {}
            self._pos = -1
            self._recording = True
            self.ops = 0
            self.faulted_ops = 0
            # OGKM_MODE_TRACE=N: remember the last N ops, printed when one fails.
            import collections
            import os

            n = int(os.environ.get("OGKM_MODE_TRACE", "0"))
            self._last = collections.deque(maxlen=n) if n > 0 else None
            self.prefetches = 0

        # ---------------------------------------------------------- mode

        def _stream(self) -> int:
            return torch.cuda.current_stream(self.device).cuda_stream

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            kwargs = kwargs or {}
            if func.is_view or func in _METADATA_OPS:
                return func(*args, **kwargs)  # no data is touched
            if func.__name__.startswith("_foreach_"):
                split = self._split_foreach(func, args, kwargs)
                if split is not _NOT_SPLIT:
                    return split
            w = self._writes.get(func)
            if w is None:
                w = self._writes[func] = _writes_of(func)
            wpos, wnames = w
            ptrs: list[tuple[int, bool]] = []

            def add(x, write: bool):
                if isinstance(x, torch.Tensor):
                    if x.device.type == "cuda" and (x.device.index or 0) == self.device:
                        p = x.untyped_storage().data_ptr()
                        if p:
                            ptrs.append((p, write))
                elif isinstance(x, (list, tuple)):
                    for y in x:
                        add(y, write)

            for i, a in enumerate(args):
                add(a, i in wpos)
            for k, a in kwargs.items():
                add(a, k in wnames)
            stream = self._stream() if ptrs else 0
            held, persistent = lib.torch_op_begin(ptrs, self.device, stream) if ptrs else ((), ())
            self.ops += 1
            if self._last is not None:
                self._last.append((self.ops, func.__name__, len(held)))
            out = None  # an op that raises allocated nothing: its holds are still dropped below
            try:
                out = func(*args, **kwargs)
            except BaseException:
                if self._last is not None:
                    import sys

                    print(f"ogkm.managed: op #{self.ops} {func.__name__} failed; previous ops: {list(self._last)}",
                          file=sys.stderr, flush=True)
                raise
            finally:
                # Outputs the op allocated hold their allocation lease: drop it.
                outs = []
                flat, _ = tree_flatten(out)
                for t in flat:
                    if isinstance(t, torch.Tensor) and t.device.type == "cuda":
                        p = t.untyped_storage().data_ptr()
                        if p:
                            outs.append(p)
                if held or outs:
                    lib.torch_op_end(held, outs, self.device, stream or self._stream())
            if held:
                self.faulted_ops += 1
            if persistent:
                # Position key: the long-lived operands (parameters / buffers);
                # activations get new addresses every pass.
                self._advance(tuple(persistent))
            return out

        # ---------------------------------------------------------- multi-tensor ops
        def _split_foreach(self, func, args, kwargs):
            """A ``_foreach_*`` op (optimizer steps, grad clipping) touches every
            parameter at once - more than the arena when the model
            oversubscribes it. Run it on consecutive slices of its lists that
            fit in half the arena instead (elementwise: same results)."""
            lens = [len(a) for a in args if isinstance(a, (list, tuple))]
            if not lens:
                return _NOT_SPLIT
            n = lens[0]
            tensors = [a for a in args if isinstance(a, (list, tuple)) and len(a) == n and n
                       and isinstance(a[0], torch.Tensor)]
            if not tensors:
                return _NOT_SPLIT
            sizes = [sum(lst[i].untyped_storage().nbytes() for lst in tensors) for i in range(n)]
            budget = max(1, self._arena_bytes() // 2)
            if sum(sizes) <= budget:
                return _NOT_SPLIT
            pieces, start, acc = [], 0, 0
            for i, sz in enumerate(sizes):
                if acc and acc + sz > budget:
                    pieces.append((start, i))
                    start, acc = i, 0
                acc += sz
            pieces.append((start, n))
            if len(pieces) == 1:
                return _NOT_SPLIT  # one tensor alone exceeds the budget: nothing to split
            outs = []
            for a0, a1 in pieces:
                sub = [a[a0:a1] if isinstance(a, (list, tuple)) and len(a) == n else a for a in args]
                outs.append(self.__torch_dispatch__(func, (), tuple(sub), kwargs))
            if all(o is None for o in outs):
                return None if outs[0] is None else outs[0]
            if isinstance(outs[0], (list, tuple)):
                return [t for o in outs for t in o]
            return outs[-1]

        def _arena_bytes(self) -> int:
            return _arena_capacity(self.device) or (1 << 62)

        # ---------------------------------------------------------- prefetch
        def _advance(self, key: tuple[int, ...]) -> None:
            """Track the position in the recorded operand sequence and prefetch
            the operands of the ops that follow."""
            if self.lookahead_bytes <= 0:
                return
            n = len(self._trace)
            nxt = self._pos + 1
            if n and nxt < n and self._trace[nxt] == key:
                self._pos = nxt
            elif key in self._first:
                self._pos = self._first[key]
                self._recording = False
            elif self._recording:
                self._first[key] = n
                self._trace.append(key)
                self._pos = n
                return
            else:
                return
            if self._recording:
                return
            want, seen, budget = [], set(key), self.lookahead_bytes
            i = self._pos + 1
            while budget > 0 and i < self._pos + 1 + len(self._trace):
                for p in self._trace[i % len(self._trace)]:
                    if p in seen:
                        continue
                    seen.add(p)
                    sz = self._sizes.get(p)
                    if sz is None:
                        sz = self._sizes[p] = lib.torch_managed_size(p, self.device)
                    budget -= sz
                    if budget < 0:
                        break
                    want.append(p)
                i += 1
            if want:
                self.prefetches += lib.torch_prefetch(want, self.device)

    _MODE_CLS = ManagedMode
    return ManagedMode


_METADATA_OPS: frozenset = frozenset()
_NOT_SPLIT = object()


def _arena_capacity(device: int) -> int:
    """Bytes of the HBM arena of ``device`` (0 before it exists)."""
    if not lib.is_initialized():
        return 0
    for a in lib.stats().get("arenas", []):
        if a["name"] == f"hbm{device}":
            return int(a["capacity"])
    return 0


def managed(device: int = 0, lookahead_bytes: Optional[int] = None):
    """Context manager: run unmodified torch code with transparent residency
    management of managed tensors (see the module docstring)."""
    global _METADATA_OPS
    import torch

    if not _METADATA_OPS:
        aten = torch.ops.aten
        _METADATA_OPS = frozenset({aten.detach.default, aten.sym_size.int, aten.sym_stride.int,
                                   aten.sym_numel.default, aten.sym_storage_offset.default})
    return _mode_class()(device=device, lookahead_bytes=lookahead_bytes)
