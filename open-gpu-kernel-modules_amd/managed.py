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

Operand geometry: an op hold covers only the pages its views of a storage
span (storage offset, sizes, strides), and a written view revokes the other
copies of exactly the 4 KB pages it writes - reads duplicate, so an evicted
tensor's host copy stays valid and only what was written since goes back
(a KV-cache row append dirties B x H pages, not the cache).

Layer-ahead prefetch and next-use eviction (the D26 prefetcher at op
granularity, with Belady replacement): the mode records the sequence of
persistent operand sets of the first pass; on later passes it recognises its
position, tells the runtime when each operand is needed next (the arena then
evicts the data needed furthest in the future instead of the least recently
used - which, on a cyclic decode step larger than HBM, is exactly the data
needed next), and prefetches the operands of the next ops (up to
``lookahead_bytes``), each allowed to evict only data needed after it.

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

    # the current stream's handle without building a torch.cuda.Stream object
    # (~2.5 us per op otherwise)
    _raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)

    def _raw_stream(device: int) -> int:
        return _raw(device) if _raw is not None else torch.cuda.current_stream(device).cuda_stream

    def _writes_of(func) -> tuple[frozenset, frozenset]:
        """(positional indices, kwarg names) of the arguments the op writes.
        aten / prims schemas declare every mutation; an op from any other
        namespace (a custom op registered without ``mutates_args``, an
        extension kernel that writes an input) is not trusted: all its tensor
        arguments count as written, so the pages it covers revoke their other
        copies - otherwise a read-mostly host duplicate would stay valid and an
        eviction would drop the GPU write."""
        pos, names = set(), set()
        trusted = getattr(func, "namespace", "aten") in ("aten", "prims")
        for i, a in enumerate(func._schema.arguments):
            if (a.alias_info is not None and a.alias_info.is_write) or not trusted:
                pos.add(i)
                names.add(a.name)
        return frozenset(pos), frozenset(names)

    class ManagedMode(TorchDispatchMode):
        device_type = "cuda"

        def __init__(self, device: int = 0, lookahead_bytes: Optional[int] = None):
            super().__init__()
            self.device = int(device)
            # default: an eighth of the arena. With next-use eviction a longer
            # window cannot push out operands needed before the prefetched ones
            # (each prefetch evicts only data needed after it, or is dropped);
            # under plain LRU anything above ~512 MB thrashed
            # (profiles/r3_managed_lookahead.txt).
            if lookahead_bytes is None:
                lookahead_bytes = _arena_capacity(self.device) // 8
            self.lookahead_bytes = int(lookahead_bytes)
            # this mode's op clock starts at 0: drop the arena's clock and the
            # hints a previous producer (another managed() context) left behind
            if lib.is_initialized():
                lib.reset_op_clock(self.device)
            self._writes: dict = {}
            self._sizes: dict[int, int] = {}
            self._trace: list[tuple[int, ...]] = []   # operand sets of the recorded pass
            self._first: dict[tuple[int, ...], int] = {}
            self._nextd: list[dict[int, int]] = []    # per position: operand -> positions to its next use
            self._pos = -1
            self._abs = 0          # op clock: trace positions passed since recording ended
            self._recording = True
            self._requested: dict[int, int] = {}  # operand -> op-clock time a prefetch was queued for
            self.ops = 0
            self.faulted_ops = 0
            self.hinted_ops = 0      # ops whose operands got next-use hints (position found in the trace)
            self.trace_misses = 0    # ops with persistent operands not found in the recorded trace
            # OGKM_MODE_TRACE=N: remember the last N ops, printed when one fails.
            import collections
            import os

            n = int(os.environ.get("OGKM_MODE_TRACE", "0"))
            self._last = collections.deque(maxlen=n) if n > 0 else None
            self.prefetches = 0

        # ---------------------------------------------------------- mode

        def _stream(self) -> int:
            return _raw_stream(self.device)

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
            operands: list = []
            dev_type = self.device_type

            def add(x, write: bool):
                if isinstance(x, torch.Tensor):
                    if x.device.type == dev_type and (x.device.index or 0) == self.device:
                        st = x.untyped_storage()
                        p = st.data_ptr()
                        if p:
                            op = _operand(x, p, st.nbytes(), write)
                            if op is not None:
                                operands.append(op)
                elif isinstance(x, (list, tuple)):
                    for y in x:
                        add(y, write)

            for i, a in enumerate(args):
                add(a, i in wpos)
            for k, a in kwargs.items():
                add(a, k in wnames)
            stream = self._stream() if operands else 0
            held, persistent = lib.torch_op_begin(operands, self.device, stream) if operands else ((), ())
            self.ops += 1
            if self._last is not None:
                self._last.append((self.ops, func.__name__, len(held)))
            out = None  # an op that raises allocated nothing: its holds are still dropped below
            done = False
            hints, want = (), ()
            try:
                out = func(*args, **kwargs)
                done = True
            except BaseException:
                if self._last is not None:
                    import sys

                    print(f"ogkm.managed: op #{self.ops} {func.__name__} failed; previous ops: {list(self._last)}",
                          file=sys.stderr, flush=True)
                raise
            finally:
                # Position in the trace (long-lived operands key it: activations
                # get new addresses every pass) -> next-use hints and prefetches.
                if persistent and done:
                    hints, want = self._advance(tuple(persistent))
                # Outputs the op allocated hold their allocation lease: drop it.
                outs = []
                if out is not None:
                    flat, _ = tree_flatten(out)
                    for t in flat:
                        if isinstance(t, torch.Tensor) and t.device.type == dev_type:
                            p = t.untyped_storage().data_ptr()
                            if p:
                                outs.append(p)
                if held or outs:
                    lib.torch_op_end(list(held), outs, self.device, stream or self._stream(), list(hints),
                                     self._abs if not self._recording else 0)
            if held:
                self.faulted_ops += 1
            if want:
                self.prefetches += lib.torch_prefetch(want, self.device)
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

        # ---------------------------------------------------------- trace / prefetch
        def _advance(self, key: tuple[int, ...]):
            """Track the position in the recorded operand sequence. Returns the
            next-use hints of this op's operands [(ptr, op clock)] and the
            prefetches to queue [(ptr, op clock it is needed at)]."""
            n = len(self._trace)
            nxt = self._pos + 1
            if n and nxt < n and self._trace[nxt] == key:
                new = nxt
            elif key in self._first:
                new = self._first[key]
                if self._recording:
                    self._recording = False
                    self._build_next_use()
            elif self._recording:
                self._first[key] = n
                self._trace.append(key)
                self._pos = n
                return (), ()
            else:
                self.trace_misses += 1
                return (), ()  # an op outside the recorded pass
            if self._recording:
                self._pos = new
                return (), ()
            step = (new - self._pos) % n if self._pos >= 0 else 0
            self._abs += step if step else n
            self._pos = new
            now = self._abs
            nd = self._nextd[new]
            # next uses only: the runtime decides keep / stream classes itself (SpreadPolicy)
            hints = [(p, now + nd[p]) for p in key]
            self.hinted_ops += 1
            want = []
            if self.lookahead_bytes > 0:
                seen, budget = set(key), self.lookahead_bytes
                for j in range(1, n + 1):
                    if budget <= 0:
                        break
                    for p in self._trace[(new + j) % n]:
                        if p in seen:
                            continue
                        seen.add(p)
                        sz = self._sizes.get(p)
                        if sz is None:
                            sz = self._sizes[p] = lib.torch_managed_size(p, self.device)
                        budget -= sz
                        if budget < 0:
                            break
                        at = now + j
                        if self._requested.get(p) != at:
                            self._requested[p] = at
                            want.append((p, at))
            return hints, want

        def _build_next_use(self) -> None:
            """For every position: positions until each operand's next use (cyclic)."""
            n = len(self._trace)
            last: dict[int, int] = {}
            nextd: list[dict[int, int]] = [dict() for _ in range(n)]
            for i in range(2 * n - 1, -1, -1):
                for p in self._trace[i % n]:
                    if i < n:
                        nextd[i][p] = last[p] - i if p in last else n
                    last[p] = i
            self._nextd = nextd

    _MODE_CLS = ManagedMode
    return ManagedMode


_METADATA_OPS: frozenset = frozenset()
_NOT_SPLIT = object()
_MAX_RUNS = 16384  # contiguous runs enumerated per written view (beyond: its bounding extent)


def _operand(x, ptr: int, nbytes: int, write: bool) -> tuple:
    """(storage ptr, write, lo, hi, written) of one tensor argument: the byte
    extent its view spans in the storage (hi == 0: all of it) and, for a
    written non-contiguous view, the 4 KB-page intervals it writes (a flat
    int64 array of [start, end) pairs; None: the whole extent). Conservative by
    construction - every byte the view can address is inside."""
    es = x.element_size()
    off = x.storage_offset() * es
    n = x.numel()
    if n == 0:
        return None  # touches nothing
    if x.is_contiguous():
        lo, hi = off, off + n * es
        if lo == 0 and hi >= nbytes:
            return (ptr, write, 0, 0, None)
        return (ptr, write, lo, hi, None)
    dims = [(s, st * es) for s, st in zip(x.shape, x.stride()) if s > 1 and st != 0]
    hi = off + sum((s - 1) * st for s, st in dims) + es
    if not write:
        return (ptr, False, off, hi, None)
    return (ptr, True, off, hi, _written_pages(off, es, dims))


def _written_pages(off: int, es: int, dims: list):
    """Page intervals (bytes, flat [start, end) pairs) addressed by a strided
    view: the innermost dims that are contiguous form runs; the runs' start
    offsets are enumerated and merged page by page. None when there are more
    than _MAX_RUNS runs (the caller then uses the bounding extent)."""
    import numpy as np

    dims = sorted(dims, key=lambda d: d[1])
    run, k = es, 0
    while k < len(dims) and dims[k][1] == run:
        run *= dims[k][0]
        k += 1
    outer = dims[k:]
    cnt = 1
    for s, _ in outer:
        cnt *= s
    if cnt > _MAX_RUNS:
        return None
    starts = np.array([off], dtype=np.int64)
    for s, st in outer:
        starts = (starts[:, None] + np.arange(s, dtype=np.int64) * st).ravel()
    p0 = np.sort(starts) >> 12
    p1 = (np.sort(starts) + (run - 1)) >> 12
    end = np.maximum.accumulate(p1)
    new = np.empty(len(p0), dtype=bool)
    new[0] = True
    new[1:] = p0[1:] > end[:-1] + 1
    idx = np.flatnonzero(new)
    lo_p = p0[idx]
    hi_p = np.append(end[idx[1:] - 1], end[-1])
    return np.stack([lo_p << 12, (hi_p + 1) << 12], axis=1).ravel()


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

    if lib.is_initialized():
        for a in lib.stats().get("arenas", []):
            t = a.get("vmm_selftest", {})
            if a["name"] == f"hbm{device}" and t.get("ran") and not t.get("ok"):
                raise RuntimeError(f"ogkm.managed(): GPU {device} failed the stable-VA translation self-test "
                                   f"({t.get('detail')}); the transparent mode would risk stale reads and is off")
    if not _METADATA_OPS:
        aten = torch.ops.aten
        _METADATA_OPS = frozenset({aten.detach.default, aten.sym_size.int, aten.sym_stride.int,
                                   aten.sym_numel.default, aten.sym_storage_offset.default})
    return _mode_class()(device=device, lookahead_bytes=lookahead_bytes)
