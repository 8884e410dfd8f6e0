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
