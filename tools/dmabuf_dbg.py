"""Debug: dma-buf export + interop import in one process, step by step."""
import faulthandler, sys, importlib
faulthandler.enable()
sys.path.insert(0, ".")
importlib.import_module("open-gpu-kernel-modules_amd")
import torch
from ogkm import rt
from ogkm._native import lib
rt.init("hip", hbm_budget={0: 1 << 30})
b = rt.alloc_device_p2p(4 << 20, 0, "exp")
info = lib.range_info(b.id)
print("ext_ptr", hex(info["ext_ptr"]), flush=True)
fd, off = lib.export_dmabuf(info["ext_ptr"], 4 << 20)
print("exported fd", fd, "off", off, flush=True)
p, n = lib.import_dmabuf(0, fd)
print("imported", hex(p), n, flush=True)
t = rt._tensor_from_ptr(p + off, (1024,), torch.int32, "cuda", 0)
print("tensor ok", flush=True)
print(t[:4].cpu(), flush=True)
lib.unimport_dmabuf(p)
print("done", flush=True)
