"""Debug: small k_fault_stress run, print the ring header while draining."""
import sys, time, importlib
sys.path.insert(0, ".")
importlib.import_module("open-gpu-kernel-modules_amd")
import torch
from ogkm import rt
from ogkm._native import lib

rt.init("hip", host_budget_mb=1024, hbm_budget={0: 1 << 30})
print("info0", lib.fault_buffer_info(0), flush=True)
gave_up = torch.zeros(1, dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()
lib.fault_stress(0, 1, 1, gave_up.data_ptr(), s.cuda_stream)   # 64 records
time.sleep(0.5)
print("after 64", lib.fault_buffer_info(0), "gave_up", int(gave_up), flush=True)
got = lib.drain_fault_records(0)
print("drained", len(got), got[:3], flush=True)
print("info", lib.fault_buffer_info(0), flush=True)
lib.fault_stress(0, 4, 32, gave_up.data_ptr(), s.cuda_stream)  # 8192 records, ring 4096
t0 = time.time()
n = 0
while time.time() - t0 < 25 and n < 8192:
    n += len(lib.drain_fault_records(0))
print("drained2", n, lib.fault_buffer_info(0), flush=True)
s.synchronize()
print("gave_up", int(gave_up), flush=True)
