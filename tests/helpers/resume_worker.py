"""save: build a TieredLlama, decode 2 steps, checkpoint it (residency map with
data + sidecar), decode one more step and keep its logits as the reference.
restore: in a fresh process, resume the model in place and decode that step.
argv: save|restore <dir> <backend fake|hip> <weight_format> <kv_format>"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from ogkm import rt  # noqa: E402
from ogkm._native import lib  # noqa: E402
from ogkm.models import llama  # noqa: E402


def main():
    mode, d, backend, wf, kf = sys.argv[1:6]
    if backend == "fake":
        rt.init("fake", fake_devices=1, fake_hbm_mb=256, host_budget_mb=1024)
        dev = "cpu"
    else:
        rt.init("hip", host_budget_mb=4096)
        dev = "cuda"
    ck = os.path.join(d, "model.json")
    if mode == "save":
        m = llama.TieredLlama(llama.CONFIGS["small"], batch=4, context=128, max_new_tokens=8, oversub=2.0,
                              lookahead=1, seed=11, weight_format=wf, kv_format=kf)
        m.keep_logits = True
        tok = torch.tensor([3, 1, 4, 1], device=dev)
        for _ in range(2):
            tok = m.step(tok)
        side = m.save(ck)
        ranges = {i: (lib.range_info(i)["addr"], lib.range_info(i)["dev_va"])
                  for i in [side["embed"], side["kv"]] + [u[1] for u in side["units"]]}
        nxt = m.step(tok)
        torch.save({"tok": tok.cpu(), "logits": m.last_logits.float().cpu(), "next": nxt.cpu(), "pos": side["pos"],
                    "ranges": ranges}, os.path.join(d, "ref.pt"))
        m.close()
    else:
        ref = torch.load(os.path.join(d, "ref.pt"), weights_only=True)
        m = llama.TieredLlama.restore(ck)
        assert m.pos == ref["pos"], (m.pos, ref["pos"])
        for i, (addr, dva) in ref["ranges"].items():
            info = lib.range_info(int(i))
            assert (info["addr"], info["dev_va"]) == (addr, dva), (i, info, addr, dva)
        m.keep_logits = True
        nxt = m.step(ref["tok"].to(dev))
        same = torch.equal(m.last_logits.float().cpu(), ref["logits"]) and torch.equal(nxt.cpu(), ref["next"])
        print(json.dumps({"identical": same, "pos": m.pos, "ranges": len(ref["ranges"])}))
        m.close()
    lib.shutdown()


if __name__ == "__main__":
    main()
