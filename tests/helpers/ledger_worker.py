"""Worker for tests/test_node_ledger.py: one rank process of an 8-GPU node on
the fake backend (its own runtime, GPU ``RANK``, host tier on that GPU's NUMA
node), sharing the node-wide ledger (OGKM_NODE_LEDGER) with the other ranks.
Writes host-resting managed data until the runtime refuses, then reports what
it got and what the ledger shows, and waits at a file barrier so every rank's
reservations are live together.

    python ledger_worker.py BARRIER_DIR WORLD
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from ogkm import rt  # noqa: E402
from ogkm._native import lib  # noqa: E402

MB = 1 << 20
bar, world = sys.argv[1], int(sys.argv[2])
rank = int(os.environ["RANK"])
rt.init("fake", fake_devices=world, fake_hbm_mb=64, local_devices=1 << rank, fake_numa_nodes=2,
        node_budget_mb=int(os.environ.get("NODE_BUDGET_MB", "96")), host_segment_mb=16)
lib.init_device(rank, 32 * MB)
node = lib.host_node()
want = int(os.environ.get("DEMAND_MB", "48"))
bufs, ok, refused, err = [], 0, 0, ""
for i in range(want // 2):
    b = rt.malloc_managed(2 * MB, f"r{rank}-{i}", cpu_view=False)
    b.set_preferred_location(rt.Loc.host(node))
    try:
        b.write(torch.full((2 * MB,), rank, dtype=torch.uint8))
        bufs.append(b)
        ok += 2 * MB
    except lib.RuntimeStatusError as e:
        refused += 1
        err = str(e)
        b.free()
        break
led = lib.node_ledger(2)
open(os.path.join(bar, f"{rank}.done"), "w").close()
t0 = time.time()
while len([f for f in os.listdir(bar) if f.endswith(".done")]) < world and time.time() - t0 < 120:
    time.sleep(0.05)
led_all = lib.node_ledger(2)  # every rank's reservations live
intact = all(bytes(b.read()[:2]) == bytes([rank, rank]) for b in bufs)
print(json.dumps({"rank": rank, "node": node, "ok_bytes": ok, "refused": refused, "error": err,
                  "ledger": led, "ledger_all": led_all, "intact": intact,
                  "refusals": lib.stats().get("ledger_refusals", 0)}), flush=True)
for b in bufs:
    b.free()
lib.shutdown()
