import sys; sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import time, torch, ogkm
from ogkm import rt
from ogkm._native import lib
rt.init("fake", fake_devices=1, fake_hbm_mb=3072, host_budget_mb=4096)
b = rt.malloc_managed(1200<<20, "w", cpu_view=False)
b.set_preferred_location(rt.Loc.gpu(0))
b.write(torch.zeros(600<<20, dtype=torch.bfloat16))
l = b.acquire(0, rt.READ); l.wait(0); l.release(0)
lib.sync_all()
t0=time.perf_counter(); n=20
for _ in range(n):
    l = b.acquire(0, rt.READ); l.wait(0); l.release(0)
dt=(time.perf_counter()-t0)/n
print(f"acquire+wait+release 1.2 GB resident: {dt*1e3:.3f} ms")
import cProfile, pstats
cProfile.run("for _ in range(10):\n    l = b.acquire(0, rt.READ); l.wait(0); l.release(0)", "/tmp/acq.prof")
pstats.Stats("/tmp/acq.prof").sort_stats("cumtime").print_stats(8)
