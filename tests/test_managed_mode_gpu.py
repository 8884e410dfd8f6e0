"""Transparent tensor-granular faults for unmodified PyTorch code
(open-gpu-kernel-modules_amd/managed.py): a stock torch.nn transformer whose
parameters exceed the HBM arena 2x runs inference and a training step under
``ogkm.managed()`` - no framework call inside the model - and its outputs,
gradients and updated parameters equal the plain (resident) run bit for bit.
Reference: the replayable fault path uvm_gpu_replayable_faults.c:2906, CPU
faults uvm.c:576, prefetch uvm_migrate.c:882 (SURVEY.md §7.1 design (1))."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "helpers", "managed_mode_worker.py")


def _run(args, tmp_path):
    r = subprocess.run([sys.executable, WORKER] + args, capture_output=True, text=True, timeout=150,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    print(r.stdout[-2000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("lazy", [True, False], ids=["lazy_unmap", "eager_unmap"])
def test_stock_transformer_oversubscribed_bitwise(tmp_path, lazy):
    import torch

    ref = tmp_path / "plain.pt"
    out = tmp_path / "managed.pt"
    _run(["plain", str(ref)], tmp_path)
    log = _run(["managed", str(out)] + (["--lazy"] if lazy else []), tmp_path)
    assert "MANAGED_OK" in log
    info = eval(log.split("MANAGED_OK", 1)[1].strip().splitlines()[0])  # noqa: S307 - our own dict repr
    assert info["param_mb"] >= 2 * info["arena_mb"], info
    assert info["evictions"] > 0 and info["vmm_errors"] == 0, info
    a = torch.load(ref, weights_only=True)
    b = torch.load(out, weights_only=True)
    assert a.keys() == b.keys()
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    assert not bad, f"{len(bad)} tensors differ, e.g. {bad[:5]}"


def test_packed_host_copies_run_bitwise_under_managed_mode(tmp_path):
    """Weights whose GPU copies were dropped clean get ANS1-packed host copies;
    the next passes refill HBM from the packed bytes (SDMA into staging, then
    k_ans_blocks on the H2D ring) and the model still matches the plain run bit
    for bit (packed copies of tensors the training step writes are expanded
    or dropped on the way)."""
    import torch

    ref = tmp_path / "plain.pt"
    out = tmp_path / "managed.pt"
    _run(["plain", str(ref)], tmp_path)
    log = _run(["managed", str(out), "--pack"], tmp_path)
    info = eval(log.split("MANAGED_OK", 1)[1].strip().splitlines()[0])  # noqa: S307 - our own dict repr
    assert info["packed_blocks"] > 0 and info["packed_decodes"] > 0, info
    a = torch.load(ref, weights_only=True)
    b = torch.load(out, weights_only=True)
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    assert not bad, f"{len(bad)} tensors differ, e.g. {bad[:5]}"


def test_accessed_by_tensors_run_bitwise_under_managed_mode(tmp_path):
    """accessed_by / preferred-host advice on managed parameters: the runtime's
    remote decision is served by a local copy (the stable VA maps HBM only)
    and the unmodified model still matches the plain run bit for bit."""
    import torch

    ref = tmp_path / "plain.pt"
    out = tmp_path / "managed.pt"
    _run(["plain", str(ref)], tmp_path)
    log = _run(["managed", str(out), "--advise"], tmp_path)
    info = eval(log.split("MANAGED_OK", 1)[1].strip().splitlines()[0])  # noqa: S307 - our own dict repr
    assert info["advised"] > 0 and info["remote_fallbacks"] > 0, info
    a = torch.load(ref, weights_only=True)
    b = torch.load(out, weights_only=True)
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    assert not bad, f"{len(bad)} tensors differ, e.g. {bad[:5]}"


OOM_SCRIPT = r"""
import os, sys
sys.path.insert(0, os.environ["OGKM_ROOT"])
import torch
from ogkm import allocator, rt
allocator.enable(managed_min_mb=1)
rt.init("hip", hbm_budget={0: 256 << 20})
keep = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
try:
    torch.empty(1 << 30, dtype=torch.uint8, device="cuda")  # 1 GB on a 256 MB arena
    print("NO_ERROR")
except (RuntimeError, MemoryError) as e:
    print("CAUGHT", type(e).__name__, "out of memory" in str(e), allocator.last_error(0) != "")
y = torch.ones(4 << 20, dtype=torch.uint8, device="cuda")  # the process carries on
torch.cuda.synchronize()
print("AFTER", int(y.sum().item()), allocator.last_error(0) == "")
"""


def test_allocation_failure_is_a_python_error():
    """An allocation the arena cannot satisfy raises in the caller (torch
    surfaces the allocator's exception as a RuntimeError) instead of aborting
    the process; later allocations still work."""
    r = subprocess.run([sys.executable, "-c", OOM_SCRIPT], capture_output=True, text=True, timeout=150,
                       env=dict(os.environ, OGKM_ROOT=os.path.dirname(HERE), HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "CAUGHT RuntimeError True True" in r.stdout or "CAUGHT MemoryError True True" in r.stdout, \
        r.stdout + r.stderr[-2000:]
    assert f"AFTER {4 << 20} True" in r.stdout, r.stdout


UNDECLARED_WRITE_SCRIPT = r"""
import os, sys
sys.path.insert(0, os.environ["OGKM_ROOT"])
import torch
import ogkm
from ogkm import allocator, rt
from ogkm._native import lib
allocator.enable(managed_min_mb=1)
rt.init("hip", hbm_budget={0: 256 << 20})
# an extension op whose schema declares no mutation but writes its input
L = torch.library.Library("ogkm_test", "DEF")
L.define("scribble(Tensor x) -> Tensor")
def _scribble(x):
    x.fill_(3)
    return x.sum(dtype=torch.int64).reshape(1)
L.impl("scribble", _scribble, "CUDA")
# 16 MB (a sum with dtype=int64 may upcast into a 128 MB temporary: it must
# fit the 256 MB arena next to the operand)
a = torch.ones(16 << 20, dtype=torch.uint8, device="cuda")
allocator.set_read_mostly(a)
with ogkm.managed():
    s0 = int(a.sum(dtype=torch.int64).item())          # read: host duplicate kept (read-mostly)
    s1 = int(torch.ops.ogkm_test.scribble(a).item())   # undeclared write
    big = [torch.full((64 << 20,), i, dtype=torch.uint8, device="cuda") for i in range(8)]  # 512 MB: a is evicted
    for b in big:
        b.add_(1)
    torch.cuda.synchronize()
    ev = lib.stats()["evictions"]
    s2 = int(a.sum(dtype=torch.int64).item())          # faulted back in: the write must have been kept
print("RESULT", s0, s1, s2, ev > 0)
"""


def test_undeclared_write_by_extension_op_survives_eviction():
    """A custom op registered without a mutation annotation writes a
    read-mostly managed tensor: the transparent mode treats operands of ops
    outside aten / prims as written, so the host duplicate is revoked and the
    eviction copies the GPU data out instead of dropping it."""
    r = subprocess.run([sys.executable, "-c", UNDECLARED_WRITE_SCRIPT], capture_output=True, text=True, timeout=150,
                       env=dict(os.environ, OGKM_ROOT=os.path.dirname(HERE), HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    n = 16 << 20
    assert f"RESULT {n} {3 * n} {3 * n} True" in r.stdout, r.stdout + r.stderr[-2000:]
