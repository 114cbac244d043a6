"""One process per GPU: rendezvous, barriers and reductions for the benchmark.

``torch.distributed`` with backend ``nccl`` (RCCL on ROCm) when GPUs are
present, ``gloo`` otherwise. Long CPU-side waits (rank 0 measuring while the
agents idle) go through a separate gloo group so no rank spins a GPU stream
in a barrier; the timed region is still bracketed by ``barrier()`` +
``torch.cuda.synchronize()`` on every rank.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Any, List, Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: Optional[torch.device] = None
    cpu_group: Any = None

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init(timeout_s: int = 1800) -> DistInfo:
    """Initialise from torchrun's env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    has_gpu = torch.cuda.is_available()
    device = None
    if has_gpu:
        torch.cuda.set_device(local % torch.cuda.device_count())
        device = torch.device("cuda", torch.cuda.current_device())
    info = DistInfo(rank=rank, world=world, local_rank=local, device=device)
    # HEADLAMP_AMD_FORCE_PG=1 builds the process groups even for one rank, so
    # the RCCL init / all-reduce path can be exercised on a single-GPU box.
    force = os.environ.get("HEADLAMP_AMD_FORCE_PG") == "1" and "MASTER_PORT" in os.environ
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "nccl" if has_gpu else "gloo"
        kw = {"device_id": device} if has_gpu else {}
        dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
        info.cpu_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s)) \
            if backend != "gloo" else None
    return info


def _active(info: DistInfo) -> bool:
    return info.world > 1 or dist.is_initialized()


def barrier(info: DistInfo) -> None:
    if _active(info):
        dist.barrier(group=info.cpu_group)


def sync_device(info: DistInfo) -> None:
    if info.device is not None:
        torch.cuda.synchronize(info.device)


def all_gather_object(info: DistInfo, obj) -> List:
    if not _active(info):
        return [obj]
    out: List = [None] * info.world
    dist.all_gather_object(out, obj, group=info.cpu_group)
    return out


def broadcast_object(info: DistInfo, obj, src: int = 0):
    if not _active(info):
        return obj
    box = [obj]
    dist.broadcast_object_list(box, src=src, group=info.cpu_group)
    return box[0]


def max_float(info: DistInfo, x: float) -> float:
    """MAX over ranks, on the device collective backend (RCCL) when present."""
    if not _active(info):
        return x
    if info.device is not None:
        t = torch.tensor([x], dtype=torch.float64, device=info.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shutdown(info: DistInfo) -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
