"""Worker for tests/test_node_ledger.py::test_concurrent_attach_on_stale_file:
attach to the node ledger the moment a start file appears (all workers race
through attach together), reserve on node 0, wait until every worker has
reserved, report the ledger, release, detach.

    python ledger_attach_worker.py BARRIER_DIR WORLD RESERVE_BYTES
    python ledger_attach_worker.py --die RESERVE_BYTES   (reserve, exit without detaching)
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from ogkm._native import lib  # noqa: E402

if sys.argv[1] == "--die":
    assert lib.ledger_attach()
    assert lib.ledger_reserve(0, int(sys.argv[2]))
    os._exit(0)  # a crashed job: slot and reservation left behind

bar, world, nbytes = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rank = int(os.environ["RANK"])


def barrier(tag: str) -> None:
    open(os.path.join(bar, f"{rank}.{tag}"), "w").close()
    t0 = time.time()
    while len([f for f in os.listdir(bar) if f.endswith("." + tag)]) < world:
        assert time.time() - t0 < 120, tag
        time.sleep(0.002)


barrier("ready")
while not os.path.exists(os.path.join(bar, "go")):
    time.sleep(0.0005)
assert lib.ledger_attach()
ok = [lib.ledger_reserve(0, nbytes) for _ in range(4)]
barrier("reserved")
view = lib.node_ledger(1)["nodes"][0]
barrier("viewed")
for k in ok:
    if k:
        lib.ledger_release(0, nbytes)
barrier("released")
after = lib.node_ledger(1)["nodes"][0]
barrier("checked")
lib.ledger_detach()
print(json.dumps({"rank": rank, "ok": ok, "view": view, "after": after}), flush=True)
