"""Worker for the collective-failure test: rank 1 never joins the second
all-reduce; rank 0's collective times out and the runtime turns sticky FATAL."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import ogkm  # noqa: E402,F401
from ogkm import rt  # noqa: E402
from ogkm._native import lib  # noqa: E402
from ogkm.parallel import comm  # noqa: E402


def main():
    e = comm.init("gloo", timeout_s=4)
    rt.init("fake", fake_devices=1, fake_hbm_mb=64, host_budget_mb=256)
    comm.all_reduce_(torch.ones(4))          # both ranks: fine
    out = {"rank": e.rank}
    if e.rank == 0:
        try:
            comm.all_reduce_(torch.ones(4))  # rank 1 never joins
            out["raised"] = False
        except comm.CollectiveError as err:
            out["raised"] = True
            out["msg"] = str(err)[:120]
        out["status"] = lib.global_status()
        out["reason"] = lib.fatal_reason()
        try:
            rt.malloc_managed(1 << 20, "after")
            out["malloc_after"] = "ok"
        except Exception as err:  # noqa: BLE001
            out["malloc_after"] = str(err)[:80]
        print("COMMFAULT " + json.dumps(out), flush=True)
        os._exit(0)
    time.sleep(12)
    os._exit(0)


if __name__ == "__main__":
    main()
