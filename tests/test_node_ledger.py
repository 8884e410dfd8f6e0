"""Node-wide host / CXL budget across rank processes (csrc/core/ledger.cpp):
the reference keeps one global pin budget for every CXL buffer in the kernel
(nv-p2p.c:1034-1111); with one runtime process per GPU the budget lives in a
shared-memory ledger every rank reserves from before it populates a host /
CXL segment."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest
import torch

from ogkm import rt
from ogkm._native import lib

HERE = os.path.dirname(os.path.abspath(__file__))
MB = 1 << 20


def _ranks(tmp_path, world: int, budget_mb: int, demand_mb: int) -> list[dict]:
    bar = tmp_path / "bar"
    bar.mkdir()
    ledger = str(tmp_path / "ledger")
    env = dict(os.environ, OGKM_NODE_LEDGER=ledger, NODE_BUDGET_MB=str(budget_mb), DEMAND_MB=str(demand_mb),
               OMP_NUM_THREADS="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "helpers", "ledger_worker.py"), str(bar), str(world)],
                              env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(world)]
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=300)
        assert p.returncode == 0, e[-3000:]
        outs.append(json.loads([l for l in o.splitlines() if l.startswith("{")][-1]))
    return outs


def test_eight_ranks_never_overcommit_a_node(tmp_path):
    """8 fake ranks on 2 NUMA nodes, each asking for 48 MB of host memory on
    its GPU's node - 192 MB per node against a 96 MB node budget. Without the
    ledger every process would size its arena at the node budget and commit
    2x the node; with it the node's reservations never pass its budget, every
    rank either gets its data or a clean NO_MEMORY, and what was written stays
    intact."""
    outs = _ranks(tmp_path, 8, 96, 48)
    by_node = {0: [], 1: []}
    for o in outs:
        by_node[o["node"]].append(o)
        assert o["intact"]
        assert o["refused"] == 0 or "NO_MEMORY" in o["error"], o
    assert len(by_node[0]) == 4 and len(by_node[1]) == 4
    # a full node's data rests on the other node (demotion), so the machine's
    # total is what bounds the ranks: 2 x 96 MB, less partly used segments
    got = sum(o["ok_bytes"] for o in outs)
    assert 2 * 96 * MB - 8 * 16 * MB <= got <= 2 * 96 * MB, got
    assert any(o["refused"] for o in outs)  # demand (384 MB) exceeded the machine: someone was refused
    for n in (0, 1):
        for o in outs:
            v = o["ledger_all"]["nodes"][n]
            assert v["capacity"] == 96 * MB and v["reserved"] <= v["capacity"], v
    assert sum(o["refusals"] for o in outs) > 0


def test_ledger_within_budget_refuses_nothing(tmp_path):
    outs = _ranks(tmp_path, 4, 256, 32)
    assert all(o["refused"] == 0 and o["ok_bytes"] == 32 * MB for o in outs), outs


def test_full_node_demotes_evictions_to_the_other_node(tmp_path, monkeypatch):
    """One process: its host node's budget is spent, so HBM evictions demote
    past it to the other node (DemotionFallbacks) instead of failing."""
    monkeypatch.setenv("OGKM_NODE_LEDGER", str(tmp_path / "ledger1"))
    if lib.is_initialized():
        lib.shutdown()
    lib.config_reset()
    # (the arena itself could hold 64 MB: the node-wide budget is what binds)
    rt.init("fake", fake_devices=2, fake_hbm_mb=64, fake_numa_nodes=2, local_devices=1, node_budget_mb=32,
            host_budget_mb=64, host_segment_mb=16)
    try:
        lib.init_device(0, 16 * MB)  # 8 chunks
        node = lib.host_node()
        filler = []
        for i in range(12):  # 24 MB resting on the host node: both 16 MB segments of its 32 MB budget
            b = rt.malloc_managed(2 * MB, f"fill{i}", cpu_view=False)
            b.set_preferred_location(rt.Loc.host(node))
            b.write(torch.zeros(2 * MB, dtype=torch.uint8))
            filler.append(b)
        hot = []
        for i in range(12):  # 24 MB of GPU-preferred data on a 16 MB arena: evictions
            b = rt.malloc_managed(2 * MB, f"hot{i}", cpu_view=False)
            b.set_preferred_location("gpu:0")
            b.write(torch.full((2 * MB,), i + 1, dtype=torch.uint8))
            hot.append(b)
        for b in hot:
            lease = b.acquire(0, rt.READ)
            lease.wait(0)
            lease.release(0)
        st = lib.stats()
        assert st["demotion_fallbacks"] > 0 and st["ledger_refusals"] > 0, st
        other = 1 - node
        on_other = [b for b in hot if any(r["tier"] == "host" and r["id"] == other
                                          for r in b.residency(0)["resident_on"])]
        assert on_other, [b.residency(0) for b in hot]
        assert [int(b.read()[0]) for b in hot] == list(range(1, 13))
        led = lib.node_ledger(2)
        assert led["nodes"][node]["reserved"] <= 32 * MB
    finally:
        lib.shutdown()
        lib.config_reset()


@pytest.mark.parametrize("round_", range(3))
def test_concurrent_attach_on_stale_file(tmp_path, round_):
    """8 processes attach at the same moment to a ledger file a crashed job left
    behind (a dead pid holding a slot and a reservation). The stale file is
    reset exactly once - no rank's reservation is wiped by another rank's
    reset - so while every rank holds its reservations the node counter equals
    the sum of the slots, and after every rank released it returns to zero
    (a release never underflows the shared counter)."""
    ledger = str(tmp_path / "ledger")
    env = dict(os.environ, OGKM_NODE_LEDGER=ledger, NODE_BUDGET_MB="4096", OMP_NUM_THREADS="1",
               OGKM_LEDGER_TEST_DELAY_US=str(20000 * round_))  # widen the scan -> reset window
    worker = os.path.join(HERE, "helpers", "ledger_attach_worker.py")
    subprocess.run([sys.executable, worker, "--die", str(300 * MB)], env=env, check=True, timeout=120)
    bar = tmp_path / "bar"
    bar.mkdir()
    world, nbytes = 8, 8 * MB
    procs = [subprocess.Popen([sys.executable, worker, str(bar), str(world), str(nbytes)],
                              env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(world)]
    import time
    t0 = time.time()
    while len([f for f in os.listdir(bar) if f.endswith(".ready")]) < world:
        assert time.time() - t0 < 240 and all(p.poll() is None for p in procs)
        time.sleep(0.01)
    (bar / "go").touch()
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e[-3000:]
        outs.append(json.loads([l for l in o.splitlines() if l.startswith("{")][-1]))
    for o in outs:
        assert all(o["ok"]), o
        # the dead job's 300 MB is gone (reset), every live rank's 4 x 8 MB counted
        assert o["view"]["reserved"] == world * 4 * nbytes, o
        assert o["view"]["mine"] == 4 * nbytes, o
        assert o["after"]["reserved"] == 0 and o["after"]["mine"] == 0, o


def test_unmatched_release_clamps_at_zero(tmp_path, monkeypatch):
    """A release without a matching reservation (e.g. made before a reset) must
    not wrap the node counter to ~2^64 and refuse every later reservation."""
    env = dict(os.environ, OGKM_NODE_LEDGER=str(tmp_path / "l2"), NODE_BUDGET_MB="64")
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from ogkm._native import lib\n"
            "assert lib.ledger_attach()\n"
            "assert lib.ledger_reserve(0, 1 << 20)\n"
            "lib.ledger_release(0, 5 << 20)\n"
            "v = lib.node_ledger(1)['nodes'][0]\n"
            "assert v['reserved'] == 0 and v['mine'] == 0, v\n"
            "assert lib.ledger_reserve(0, 32 << 20)\n"
            "lib.ledger_detach()\n") % os.path.dirname(HERE)
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=120)
