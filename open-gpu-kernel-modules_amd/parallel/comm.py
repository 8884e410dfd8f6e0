"""Process-group bootstrap and collectives: one process per GPU, RCCL over xGMI.

``torch.distributed`` with backend ``nccl`` IS RCCL on ROCm; ``gloo`` is used for
CPU runs (fake backend, tests). The reference has no collective library at all
 - these are new components the multi-GPU configs need.

xGMI is point-to-point (7 links x ~153 GB/s per GPU on an 8-GPU node): a ring
collective is bound by one link per hop, so large transfers are bucketed into a
few big messages (RCCL then spreads them over its channels), and decode-size
all-reduces (B x dim, ~1 MB) are latency-bound - they are issued back-to-back
on the compute stream without extra host synchronisation.
"""
from __future__ import annotations

import datetime
import functools
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


class CollectiveError(RuntimeError):
    """A collective failed or timed out; the runtime's status is now FATAL."""


def _fatal_on_error(fn):
    """Collective failures (peer lost, RCCL error, timeout) become the runtime's
    sticky fatal status - the analogue of a channel error setting the global
    fatal error (uvm_channel.c:2080-2112, uvm_global.c:420-438): every later
    runtime call then fails fast instead of hanging on a dead peer."""

    @functools.wraps(fn)
    def wrapper(*a, **kw):
        try:
            return fn(*a, **kw)
        except CollectiveError:
            raise
        except Exception as e:  # noqa: BLE001 - any backend error is fatal for the job
            why = f"collective {fn.__name__} failed on rank {env().rank}: {type(e).__name__}: {e}"
            try:
                from .._native import lib
                if lib.is_initialized():
                    lib.set_fatal(why[:200])
            except Exception:
                pass
            raise CollectiveError(why) from e
    return wrapper


@dataclass
class DistEnv:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    forced: bool = False  # a one-rank process group (OGKM_DIST_FORCE=1): collectives still run

    @property
    def is_dist(self) -> bool:
        return self.world > 1 or self.forced


_ENV: Optional[DistEnv] = None

# Bytes this rank receives over the links per collective kind (the xGMI traffic
# a plan predicts): a ring all-reduce of n bytes moves 2 (W-1)/W n in and out
# of every rank; an all-gather receives the other W-1 shards.
STATS = {"allreduce_bytes_in": 0, "allgather_bytes_in": 0, "collectives": 0}


def reset_stats() -> None:
    for k in STATS:
        STATS[k] = 0


def _count(kind: str, nbytes: float) -> None:
    STATS[kind] += int(nbytes)
    STATS["collectives"] += 1


def init(backend: Optional[str] = None, timeout_s: int = 600) -> DistEnv:
    """Initialise from torchrun-style env vars (RANK / WORLD_SIZE / LOCAL_RANK /
    MASTER_ADDR / MASTER_PORT). Single-process runs get a trivial env, unless
    ``OGKM_DIST_FORCE=1``: then a one-rank process group is created and every
    collective really runs (RCCL on a single GPU - the multi-GPU code path,
    stream interplay included, exercised on a one-GPU box)."""
    global _ENV
    if _ENV is not None:
        return _ENV
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    forced = world == 1 and os.environ.get("OGKM_DIST_FORCE", "0") == "1"
    if world <= 1 and not forced:
        _ENV = DistEnv(0, 1, 0, "none")
        return _ENV
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if backend == "nccl":
        # RCCL errors / timeouts are raised in the waiting thread (and abort the
        # communicator) instead of hanging the job.
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s),
                                device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
    _ENV = DistEnv(rank, world, local, backend, forced)
    return _ENV


def env() -> DistEnv:
    return _ENV if _ENV is not None else init()


def shutdown() -> None:
    global _ENV
    if _ENV is not None and _ENV.is_dist and dist.is_initialized():
        dist.destroy_process_group()
    _ENV = None


@_fatal_on_error
def barrier() -> None:
    e = env()
    if e.is_dist:
        if e.backend == "nccl":
            dist.barrier(device_ids=[e.local_rank])
        else:
            dist.barrier()


@_fatal_on_error
def all_reduce_(t: torch.Tensor) -> torch.Tensor:
    e = env()
    if e.is_dist:
        dist.all_reduce(t)
        _count("allreduce_bytes_in", 2 * (e.world - 1) / e.world * t.numel() * t.element_size())
    return t


@_fatal_on_error
def all_gather_cat(t: torch.Tensor, dim: int = 0) -> torch.Tensor:
    e = env()
    if not e.is_dist:
        return t
    out = [torch.empty_like(t) for _ in range(e.world)]
    dist.all_gather(out, t.contiguous())
    _count("allgather_bytes_in", (e.world - 1) * t.numel() * t.element_size())
    return torch.cat(out, dim=dim)


@_fatal_on_error
def all_gather_into(out: torch.Tensor, shard: torch.Tensor) -> torch.Tensor:
    """out = concat of every rank's ``shard`` (equal sizes), in rank order. RCCL:
    one all_gather_into_tensor on the current stream (the host does not wait)."""
    e = env()
    if not e.is_dist:
        out[:shard.numel()].copy_(shard.reshape(-1))
        return out
    if e.backend == "nccl":
        dist.all_gather_into_tensor(out, shard)
    else:  # gloo: list form; chunks of the flat output are 1-D, so is the shard
        dist.all_gather(list(out.reshape(-1).chunk(e.world)), shard.reshape(-1).clone())
    _count("allgather_bytes_in", (e.world - 1) * shard.numel() * shard.element_size())
    return out


@_fatal_on_error
def all_gather_objects(obj) -> list:
    """One picklable object per rank, in rank order (host-side metadata only)."""
    e = env()
    if not e.is_dist:
        return [obj]
    out = [None] * e.world
    dist.all_gather_object(out, obj)
    return out


@_fatal_on_error
def max_over_ranks(x: float) -> float:
    """Max of a host scalar over ranks (timing: the job is as slow as its slowest rank)."""
    e = env()
    if not e.is_dist:
        return x
    dev = f"cuda:{e.local_rank}" if e.backend == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
