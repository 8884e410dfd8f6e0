"""xGMI peer-migration plane on the fake backend (4 GPUs): GPU->GPU copies are
pushed by the SOURCE GPU's ring (uvm_va_block.c:3390-3460), large copies are
split over the SDMA engines of that (peer, source) pair - per-pair masks as
hsa_amd_memory_copy_engine_status(dst, src) reports them, the per-pair caps
read at uvm_gpu.c:2332-2388 - the CU push kernel (k_peer_push) is the
alternative engine, and a pair with no peer path stages through host memory
(uvm_va_block.c:4703-4836)."""
from __future__ import annotations

import pytest
import torch

from ogkm import rt
from ogkm._native import lib

MB = 1 << 20


@pytest.fixture
def fake4():
    if lib.is_initialized():
        lib.shutdown()
    lib.config_reset()
    lib.clear_fatal_for_test()
    yield
    if lib.is_initialized():
        lib.shutdown()
    lib.config_reset()


def _init(**cfg):
    for k, v in cfg.items():
        lib.configure(k, v)
    rt.init("fake", fake_devices=4, fake_hbm_mb=128, lock_check=1, host_budget_mb=1024)
    lib.reset_lock_violations()


def _bits(mask):
    return [b for b in range(32) if (mask >> b) & 1]


def test_engine_masks_are_per_pair(fake4):
    _init()
    assert lib.copy_engine_mask(0, -1) == 0x1 and lib.copy_engine_mask(-1, 0) == 0x2
    masks = {(d, s): lib.copy_engine_mask(d, s) for d in range(4) for s in range(4) if d != s}
    assert all(len(_bits(m)) == 2 for m in masks.values())
    assert masks[(1, 0)] != masks[(2, 0)]                       # engines differ per destination
    assert all(m & 0x3 == 0 for m in masks.values())            # never the host-direction engines
    assert lib.copy_engine_mask(2, 2) == 0


def test_split_over_engines_plan():
    mask = 0b1011000
    out = lib.split_over_engines([(0x100000000, 0x200000000, 64 * MB)], mask, 8 * MB)
    assert len(out) == 3 and sum(p[2] for p in out) == 64 * MB
    assert sorted(p[3] for p in out) == sorted(1 << b for b in _bits(mask))
    assert all(p[0] - 0x100000000 == p[1] - 0x200000000 for p in out)   # dst / src offsets move together
    assert all((p[0] - 0x100000000) % (64 << 10) == 0 for p in out)
    small = lib.split_over_engines([(0, 0, 4 * MB)] * 6, mask, 8 * MB)  # small copies rotate over engines
    assert [p[3] for p in small] == [1 << b for b in (_bits(mask) * 2)]
    assert lib.split_over_engines([(0, 0, 4 * MB)], 0, 8 * MB)[0][3] == 0  # no engines: unchanged


def test_peer_copy_pushed_by_source_over_pair_engines(fake4):
    _init(peer_split_min_mb=2)
    b = rt.malloc_managed(16 * MB, "peer")
    ref = torch.arange(4 * MB, dtype=torch.int32)
    b.write(ref)
    b.migrate("gpu:1")
    before = {d: lib.engine_bytes(d) for d in range(4)}
    b.migrate("gpu:3")
    after = {d: lib.engine_bytes(d) for d in range(4)}
    delta = {d: [a - c for a, c in zip(after[d], before[d])] for d in range(4)}
    mask = lib.copy_engine_mask(3, 1)
    moved = {e: delta[1][e] for e in _bits(mask)}
    assert sum(moved.values()) == 16 * MB, delta[1]              # all on GPU 1 (the source) ...
    assert all(v > 0 for v in moved.values()), moved             # ... split over both pair engines
    assert sum(delta[3]) == 0 and sum(delta[0]) == 0             # the destination issued nothing
    assert ("gpu", 3) in [(r["tier"], r["id"]) for r in b.residency(0)["resident_on"]]
    assert torch.equal(b.read().view(torch.int32), ref)
    assert lib.lock_violations() == 0
    b.free()


def test_peer_push_kernel_engine(fake4):
    _init(peer_copy_engine=0)
    b = rt.malloc_managed(8 * MB, "push")
    ref = torch.arange(2 * MB, dtype=torch.int32) * 3
    b.write(ref)
    b.migrate("gpu:2")
    push0 = lib.engine_bytes(2)[31]
    b.migrate("gpu:0")
    assert lib.engine_bytes(2)[31] - push0 == 8 * MB             # k_peer_push issued by the source (GPU 2)
    assert sum(lib.engine_bytes(2)[2:31]) == 0                   # no SDMA peer engine used
    assert torch.equal(b.read().view(torch.int32), ref)
    b.free()


def test_peer_copy_staged_through_host_without_link(fake4):
    _init()
    b = rt.malloc_managed(4 * MB, "staged")
    ref = torch.full((MB,), 7, dtype=torch.int32)
    b.write(ref)
    b.migrate("gpu:1")
    d2h0 = lib.stats()["bytes_xfer_dth"]
    lib.inject("peer_link_down", 1 << 1)                         # GPU 1 has no peer path
    b.migrate("gpu:2")
    assert lib.stats()["bytes_xfer_dth"] - d2h0 >= 4 * MB        # bounced through host memory
    assert torch.equal(b.read().view(torch.int32), ref)
    b.free()
