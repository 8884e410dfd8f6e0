import sys, importlib; sys.path.insert(0, "."); importlib.import_module("open-gpu-kernel-modules_amd")
import torch, ogkm
from ogkm import rt
from ogkm._native import lib
rt.init("hip", host_budget_mb=1024, hbm_budget={0: 1 << 30})
lib.set_log_level(3)
n = 4096
ref = torch.randint(0, 255, (n,), dtype=torch.uint8)
b = rt.malloc_managed(n, "rt")
b.write(ref)
print("residency", b.residency(0)["resident_on"])
l = b.acquire(0, rt.READ)
print("lease dptr", hex(l.dptr))
l.wait()
t = l.tensor((n,), torch.uint8)
torch.cuda.synchronize()
print("equal", torch.equal(t.cpu(), ref), t[:8].tolist(), ref[:8].tolist())
l.release()
st = lib.stats()
print({k: v for k, v in st.items() if "ring" in k or "xfer" in k})
