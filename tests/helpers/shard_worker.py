"""Worker for the peer-shard weight test (gloo, fake backend): every rank owns
half of each layer; the pipeline all-gathers layers with look-ahead and each
rank checks the gathered tensors against the full reference weights."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import ogkm  # noqa: E402,F401
from ogkm import rt  # noqa: E402
from ogkm.parallel import comm, shards  # noqa: E402


def main():
    e = comm.init("gloo")
    rt.init("fake", fake_devices=1, fake_hbm_mb=64, host_budget_mb=256)
    specs = [shards.LayerSpec(["wq", "w1"], [(33, 17), (17, 9)]),
             shards.LayerSpec(["wo"], [(65, 31)]),
             shards.LayerSpec(["a", "b", "c"], [(7,), (128, 3), (5, 5)])]
    g = torch.Generator().manual_seed(7)
    full = [{nm: torch.randn(shp, generator=g).to(torch.bfloat16) for nm, shp in zip(s.names, s.shapes)}
            for s in specs]
    sw = shards.ShardedWeights(specs, torch.bfloat16)
    for i in range(len(specs)):
        sw.load_named(i, full[i])
    pipe = shards.ShardGatherPipeline(sw, depth=2)
    ok = True
    for rep in range(2):
        for k in range(len(specs)):
            lay = pipe.get(k)
            for nm in specs[k].names:
                ok &= bool(torch.equal(lay[nm], full[k][nm]))
    pipe.drain()
    res = {"rank": e.rank, "ok": ok, "gathers": pipe.stats["gathers"], "shard_bytes": sw.shard_bytes()}
    sw.free()
    allres = [None] * e.world
    torch.distributed.all_gather_object(allres, res)
    if e.rank == 0:
        for r in allres:
            print("SHARDRESULT " + json.dumps(r), flush=True)
    comm.shutdown()


if __name__ == "__main__":
    main()
