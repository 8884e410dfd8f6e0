"""open-gpu-kernel-modules_amd: an MI355X-native unified-memory + CXL tiering
framework with the capabilities of CXLMemUring/open-gpu-kernel-modules
(nvidia-uvm fault-driven migration, nvidia-peermem P2P, the CXL fork's pool
mapping), re-designed for gfx950 / ROCm / RCCL over xGMI.

The directory name is not a Python identifier, so the package is also
registered as ``ogkm`` (``import ogkm`` after putting the repo root on
sys.path, or ``importlib.import_module("open-gpu-kernel-modules_amd")``).

Layout
  _native      native core loader (C++/HIP runtime, csrc/)
  rt           managed memory API (malloc_managed / mem_advise / mem_prefetch_async / leases)
  cxl          CXL.mem tier (discovery, registration, async DMA, bandwidth)
  tools        event queues + counters (UVM tools analog)
  checkpoint   residency-map checkpoint format
  allocator    PyTorch pluggable allocator on the HBM arena
  managed      transparent mode: tensor-granular software faults for unmodified torch code
  p2p          peer-memory client: pinned exports, dma-buf, IPC (nvidia-peermem analog)
  ops/         HIP kernel entry points (copies, managed gather) + decode ops
  models/      Llama-3 decode engine with tiered (oversubscribed) weights
  parallel/    RCCL comm, tensor parallel, peer-shard weights, topology
  diag         hang diagnostics: SIGUSR1 / watchdog dumps of every thread's stack + the runtime's rings and leases
"""
from __future__ import annotations

import sys as _sys

__version__ = "0.1.0"

from . import _native  # noqa: E402,F401  (fails loudly if the native core is missing)
from . import rt, tools, checkpoint, cxl, allocator, p2p, diag  # noqa: E402,F401
from .managed import managed  # noqa: E402,F401
from . import ops, parallel, models  # noqa: E402,F401

# Register the importable alias "ogkm" for the package and every loaded submodule.
_sys.modules.setdefault("ogkm", _sys.modules[__name__])
for _k in list(_sys.modules):
    if _k.startswith(__name__ + "."):
        _sys.modules.setdefault("ogkm." + _k[len(__name__) + 1:], _sys.modules[_k])
