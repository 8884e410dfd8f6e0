"""Worker for the multi-process model tests (gloo, fake backend): tensor
parallel (PARALLEL=tp) or peer-shard weights (PARALLEL=shards).

Launched by torch.distributed.run; rank 0 prints one JSON line with the logits
of each decode step (all sequences, full vocab), for comparison with the
single-process run."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import ogkm  # noqa: E402,F401
from ogkm import rt  # noqa: E402
from ogkm.models import llama  # noqa: E402
from ogkm._native import lib  # noqa: E402
from ogkm.parallel import comm  # noqa: E402


def main():
    e = comm.init("gloo")
    rt.init("fake", fake_devices=1, fake_hbm_mb=512, host_budget_mb=2048)
    par = os.environ.get("PARALLEL", "tp")
    batch = int(os.environ.get("BATCH", "2"))
    oversub = float(os.environ.get("OVERSUB", "1.2"))
    cfg = llama.CONFIGS[os.environ.get("MODEL", "tiny")]
    m = llama.TieredLlama(cfg, batch=batch, context=8, max_new_tokens=4, oversub=oversub, lookahead=1,
                          tp_rank=e.rank, tp_world=e.world, seed=5, parallel=par)
    m.keep_logits = True
    out = []
    for s in range(3):  # fixed input schedule: comparisons do not depend on near-tie argmax
        glob = torch.tensor([3 + s + 8 * j for j in range(batch)])
        tok = m.step(glob[m.b0:m.b0 + m.B])
        out.append({"tokens": tok.tolist(), "logits": m.last_logits[:, :64].tolist(),
                    "gathers": m.gather.stats["gathers"] if m.gather else 0})
    out.append({"host_node": lib.host_node(), "gathers": m.gather.stats["gathers"] if m.gather else 0,
                "cache_hits": m.gather.stats["cache_hits"] if m.gather else 0,
                "cache_bytes": m.gather_cache_bytes})
    if e.rank == 0:
        print("TPRESULT " + json.dumps(out), flush=True)
    m.close()
    comm.shutdown()
    rt.shutdown()


if __name__ == "__main__":
    main()
