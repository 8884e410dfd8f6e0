"""Small helpers: logging, timing, environment."""
from __future__ import annotations

import logging
import os
import time
from contextlib import contextmanager

log = logging.getLogger("ogkm")
if not log.handlers:
    _h = logging.StreamHandler()
    _h.setFormatter(logging.Formatter("[ogkm %(levelname)s] %(message)s"))
    log.addHandler(_h)
    log.setLevel(os.environ.get("OGKM_LOG", "WARNING").upper())


@contextmanager
def timed(label: str, sync_cuda: bool = True, sink: dict | None = None):
    """Wall-clock a region (synchronising the GPU on both sides when requested)."""
    import torch

    if sync_cuda and torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    yield
    if sync_cuda and torch.cuda.is_available():
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if sink is not None:
        sink[label] = dt
    log.info("%s: %.3f ms", label, dt * 1e3)


def env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return default if v is None or v == "" else int(v)
