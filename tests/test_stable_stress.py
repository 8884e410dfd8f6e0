"""Adversarial stress of the stable-VA managed path on the fake backend
("test with adversarial access patterns").

Managed tensors cycle through an arena far smaller than them. Every "op"
holds a random operand set (torch_op_begin), enqueues a lagging "kernel" on a
fake stream that reads and writes every page of those operands through their
stable VAs, and drops the holds (torch_op_end) - so the host runs far ahead of
the stream, exactly like torch ahead of the GPU. Evictions, batch copy-outs,
remaps (a block returning to another chunk), stale-mapping teardown and frees
all happen while earlier kernels are still queued. The fake backend's VMM is
real: an unmapped VA is PROT_NONE, so a mapping torn down before its last
queued user ran crashes the worker (the GPU "illegal memory access"); every
write is counted and checked at the end (a lost update = an ordering bug,
e.g. a fresh chunk written before its previous owner's copy-out finished);
and the fake backend's race detector reports any engine copy that overlaps a
kernel on the same chunk. Runs in a subprocess so a crash fails the test
instead of killing pytest."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import ctypes, random, sys
sys.path.insert(0, %r)
import ogkm
from ogkm import rt
from ogkm._native import lib
MB = 1 << 20
rt.init("fake", fake_devices=1, fake_hbm_mb=256)
lib.configure("hbm_provider", 1)
lib.configure("torch_alloc_managed_min_mb", 1)
lib.configure("stable_lazy_unmap", %d)
lib.configure("stable_batch_blocks", %d)
lib.configure("fake_race_check", 1)  # engine copy vs kernel on one chunk -> "[fake RACE]" on stderr
lib.inject("tlb_mode", %d)  # 1: a remapped VA serves its old chunk until a translation flush
lib.init_device(0, 24 * MB)  # 12 chunks
PREFETCH = %d  # asynchronous op-trace prefetches between ops (the prefetch worker remaps concurrently)
HINTS = %d  # next-use hints on every op: Belady victims and home-chunk placement (ChunkArena::reserve_for)
if PREFETCH:
    lib.configure("torch_async_prefetch", 1)
s = lib.debug_stream_create(0)
rng = random.Random(%d)
live = []
touches = {}
def alloc():
    n = rng.choice([2, 4, 6]) * MB
    held, _ = lib.torch_op_begin([], 0, s)
    p = lib.torch_alloc(n, 0, s)
    assert p, "alloc failed"
    lib.debug_stream_sync(s)
    ctypes.memset(p, 0, n)  # known start (torch ranges are not zero-filled)
    lib.debug_touch(s, p, n, 50)
    lib.torch_op_end(held, [p], 0, s)
    live.append((p, n))
    touches[p] = 1
for _ in range(6):
    alloc()
for it in range(%d):
    k = rng.randint(1, 2)
    ops = rng.sample(live, k)
    ws = [rng.random() < 0.5 for _ in ops]
    held, _ = lib.torch_op_begin([(p, w) for (p, _), w in zip(ops, ws)], 0, s)
    for (p, n), w in zip(ops, ws):
        # an operand declared read-only is only read (a read lease may keep
        # host duplicates valid): only writers count
        lib.debug_touch(s, p, n, rng.choice([0, 100, 400]), w)
        touches[p] += int(w)
    if HINTS:
        lib.torch_op_end(held, [], 0, s, [(p, it + 1 + rng.randint(0, 40)) for p, _ in ops], it + 1)
    else:
        lib.torch_op_end(held, [], 0, s)
    if PREFETCH and rng.random() < 0.6:
        lib.torch_prefetch([(q, it + 1 + rng.randint(0, 40) if HINTS else 0)
                            for q, _ in rng.sample(live, min(2, len(live)))], 0)
    r = rng.random()
    if r < 0.1 and len(live) > 4:
        p, n = live.pop(rng.randrange(len(live)))
        lib.torch_free(p, 0, s)
        del touches[p]
    elif r < 0.2:
        alloc()
lib.debug_stream_sync(s)
# Data check: every touch added 1 to the first word of every page of its
# operands (no update may be lost to an eviction / fill / remap race).
bad = 0
for p, n in live:
    held, _ = lib.torch_op_begin([(p, False)], 0, s)
    lib.debug_stream_sync(s)
    words = [ctypes.c_uint32.from_address(p + o).value for o in range(0, n, 4096)]
    lib.torch_op_end(held, [], 0, s)
    if set(words) != {touches[p]}:
        bad += 1
        print("DATA_MISMATCH", hex(p), n, touches[p], sorted(set(words))[:8])
assert bad == 0, bad
own = lib.check_ownership()  # every residency's chunk owned by its block, none shared
assert own == "", own[:2000]
st = rt.stats()
print("STRESS_OK", st["evictions"], st["vmm_remaps"], st["tlb_flushes"], st["vmm_errors"])
'''


@pytest.mark.parametrize("lazy,batch,seed,tlb,prefetch,hints", [(0, 32, 1, 0, 0, 0), (1, 32, 2, 0, 0, 0), (0, 1, 3, 0, 0, 0),
                                                               (1, 2, 4, 0, 0, 0), (0, 32, 5, 1, 1, 0), (1, 2, 6, 1, 1, 0),
                                                               (0, 4, 7, 0, 1, 0), (1, 32, 8, 1, 0, 1), (0, 4, 9, 1, 1, 1),
                                                               (1, 2, 10, 0, 1, 1)])
def test_stable_va_stress_async_users(lazy, batch, seed, tlb, prefetch, hints):
    """tlb=1: the fake translation model of gfx950 VMM - a lost update means a
    kernel ran on a stale mapping (a flush missing or not yet complete);
    prefetch=1: the asynchronous prefetch worker evicts / remaps / flushes
    concurrently with the dispatching thread's op holds."""
    code = WORKER % (ROOT, lazy, batch, tlb, prefetch, hints, seed, 300)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, f"rc={r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}"
    assert "STRESS_OK" in r.stdout
    assert "[fake RACE]" not in r.stderr, r.stderr[-3000:]
    ev, remaps, flushes, errors = map(int, r.stdout.split("STRESS_OK")[1].split()[:4])
    assert ev > 50 and remaps > 0 and errors == 0, r.stdout


@pytest.mark.parametrize("seed,prefetch", [(201, 0), (204, 1), (213, 1)])
def test_stable_va_stress_packed_merged_refills(seed, prefetch):
    """The same adversarial run with refills from ANS1-packed host copies staged
    through a small HBM staging buffer, slow decodes (the fake decode kernel
    sleeps 2 ms) and the H2D worker merging queued decode batches - the
    configuration of the transparent-mode gradient corruption bisected in
    profiles/r6_ring_merge_fix (not reproduced here, on the fake backend)."""
    extra = ('lib.configure("ring_merge_packed_mb", 64)\nlib.configure("ans_stage_mb", 8)\n'
             'lib.configure("fake_kernel_delay_us", 2000)\n')
    code = WORKER % (ROOT, seed % 2, [1, 2, 4, 32][seed % 4], (seed // 2) % 2, prefetch, (seed // 4) % 2, seed, 600)
    code = code.replace('lib.configure("fake_race_check", 1)', 'lib.configure("fake_race_check", 1)\n' + extra)
    code = code.replace('print("STRESS_OK"', 'print("PACKED", st["packed_decodes"])\nprint("STRESS_OK"')
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, f"rc={r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}"
    assert "STRESS_OK" in r.stdout
    assert int(r.stdout.split("PACKED")[1].split()[0]) > 0, r.stdout  # refills did come from packed copies
    assert "[fake RACE]" not in r.stderr, r.stderr[-3000:]
