"""Worker for the multi-process tensor-parallel test (gloo, fake backend).

Launched by torch.distributed.run; prints one JSON line per rank with the
logits of each decode step, for comparison with the single-process run."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import ogkm  # noqa: E402,F401
from ogkm import rt  # noqa: E402
from ogkm.models import llama  # noqa: E402
from ogkm.parallel import comm  # noqa: E402


def main():
    e = comm.init("gloo")
    rt.init("fake", fake_devices=1, fake_hbm_mb=512, host_budget_mb=2048)
    cfg = llama.CONFIGS["tiny"]
    m = llama.TieredLlama(cfg, batch=2, context=8, max_new_tokens=4, oversub=1.2, lookahead=1,
                          tp_rank=e.rank, tp_world=e.world, seed=5)
    m.keep_logits = True
    out = []
    for s in range(3):  # fixed input schedule: comparisons do not depend on near-tie argmax
        tok = m.step(torch.tensor([3 + s, 11 + s]))
        out.append({"tokens": tok.tolist(), "logits": m.last_logits[:, :64].tolist()})
    if e.rank == 0:
        print("TPRESULT " + json.dumps(out), flush=True)
    m.close()
    comm.shutdown()
    rt.shutdown()


if __name__ == "__main__":
    main()
