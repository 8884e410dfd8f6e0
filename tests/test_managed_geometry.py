"""The transparent mode's operand geometry (open-gpu-kernel-modules_amd/managed.py
``_operand``): the byte extent an op hold covers and the 4 KB pages a written
view dirties must contain every byte the view can address (a missed page would
leave a stale host copy marked valid), and should not be much larger. Checked
against brute-force enumeration of the element addresses of many views.
Also: an op that raises inside the mode still drops its holds."""
from __future__ import annotations

import numpy as np
import pytest
import torch
from torch.utils._python_dispatch import TorchDispatchMode

import sys

import ogkm

mm = sys.modules[ogkm.__name__ + ".managed"]


def _addresses(x: torch.Tensor) -> np.ndarray:
    es = x.element_size()
    idx = np.zeros(1, dtype=np.int64) + x.storage_offset()
    for s, st in zip(x.shape, x.stride()):
        idx = (idx[:, None] + np.arange(s, dtype=np.int64) * st).ravel()
    return idx * es


def _pages_of(intervals) -> set:
    out = set()
    for lo, hi in zip(intervals[0::2], intervals[1::2]):
        assert lo % 4096 == 0 and hi % 4096 == 0 and hi > lo
        out.update(range(lo >> 12, hi >> 12))
    return out


VIEWS = [
    lambda b: b[:, :, 5],                      # KV-cache row append [B, H, T, hd] -> [B, H, hd]
    lambda b: b[:, :, :9],                     # prefix read
    lambda b: b[1:3],                          # contiguous slice
    lambda b: b.transpose(0, 2),               # permuted
    lambda b: b[:, 1, ::3],                    # strided
    lambda b: b[..., 7],                       # one element per row
    lambda b: b[2, :, 4:6],
    lambda b: b.reshape(-1)[100:5000],
    lambda b: b.reshape(-1)[::4097],
    lambda b: b[:, :, 3:4].expand(-1, -1, 6, -1),  # broadcast (stride 0)
]


@pytest.mark.parametrize("k", range(len(VIEWS)))
@pytest.mark.parametrize("write", [False, True])
def test_operand_extent_covers_every_addressed_byte(k, write):
    base = torch.zeros(6, 8, 64, 96, dtype=torch.bfloat16)  # 6 MB storage
    x = VIEWS[k](base)
    st = base.untyped_storage()
    op = mm._operand(x, 4096, st.nbytes(), write)
    assert op is not None
    ptr, w, lo, hi, written = op
    assert ptr == 4096 and w == write
    addr = _addresses(x)
    a0, a1 = int(addr.min()), int(addr.max()) + x.element_size()
    if hi == 0:
        assert lo == 0  # the whole storage
    else:
        assert lo <= a0 and a1 <= hi
        assert hi - lo <= a1 - a0 + 4096  # the bounding extent, not more
    if write and written is not None:
        pages = _pages_of(list(written))
        need = set((addr >> 12).tolist()) | set(((addr + x.element_size() - 1) >> 12).tolist())
        assert need <= pages
        assert pages == need  # exactly the touched pages


def test_kv_row_append_dirties_only_its_pages():
    kv = torch.zeros(64, 8, 1024, 128, dtype=torch.bfloat16)  # 128 MB, the stock 8B's per-layer K cache
    op = mm._operand(kv[:, :, 700], 1 << 40, kv.untyped_storage().nbytes(), True)
    pages = _pages_of(list(op[4]))
    assert len(pages) == 64 * 8  # one 4 KB page per (sequence, head): 2 MB dirty, not 128 MB


def test_empty_view_touches_nothing():
    b = torch.zeros(16, 16)
    assert mm._operand(b[3:3], 4096, b.untyped_storage().nbytes(), True) is None


def test_op_that_raises_drops_its_holds(monkeypatch):
    """Every hold torch_op_begin took is dropped by torch_op_end even when the
    op raises, and the op's own exception reaches the caller."""
    calls = []
    monkeypatch.setattr(mm.lib, "torch_op_begin", lambda ops, dev, stream: (([o[0] for o in ops]), ()),
                        raising=False)
    monkeypatch.setattr(mm.lib, "torch_op_end", lambda held, outs, *a: calls.append((list(held), list(outs))),
                        raising=False)
    m = ogkm.managed(lookahead_bytes=0)
    m.device_type = "cpu"
    m._stream = lambda: 0
    a, b = torch.randn(4, 5), torch.randn(3, 7)
    TorchDispatchMode.__enter__(m)
    try:
        with pytest.raises(RuntimeError, match="shapes cannot be multiplied|size mismatch|mat1 and mat2"):
            torch.mm(a, b)
    finally:
        TorchDispatchMode.__exit__(m, None, None, None)
    assert calls and calls[-1][0] == [a.untyped_storage().data_ptr(), b.untyped_storage().data_ptr()]
    assert calls[-1][1] == []


def test_trace_next_use_distances():
    m = ogkm.managed(lookahead_bytes=0)
    m._trace = [(1, 2), (3,), (1,), (4, 2)]
    m._build_next_use()
    assert m._nextd[0] == {1: 2, 2: 3}
    assert m._nextd[1] == {3: 4}
    assert m._nextd[2] == {1: 2}
    assert m._nextd[3] == {4: 4, 2: 1}
