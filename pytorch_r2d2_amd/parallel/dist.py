"""Process-group setup (one process per GPU; RCCL over xGMI on MI355X, gloo on CPU).

The reference has no torch.distributed at all: learner -> actors weights go through
a ``multiprocessing.Manager`` dict and experience through pickle files.  Here every
cross-process byte on the GPU path rides ``torch.distributed`` with backend ``nccl`` (which IS
RCCL on ROCm); CPU tests use ``gloo`` with the same code.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def init_distributed(backend: str = "auto", timeout_s: float = 600.0,
                     device_type: Optional[str] = None) -> DistInfo:
    """Initialise from torchrun-style env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).
    With WORLD_SIZE<=1 nothing is initialised.  MASTER_ADDR defaults to 127.0.0.1."""
    world = env_world()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = torch.cuda.is_available() if device_type is None else device_type == "cuda"
    if backend == "auto":
        backend = "nccl" if use_gpu else "gloo"
    device = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
    if world <= 1:
        return DistInfo(0, 1, 0, "none", device)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if not dist.is_initialized():
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return DistInfo(dist.get_rank(), dist.get_world_size(), local, backend, device)


def barrier(info: Optional[DistInfo] = None):
    if dist.is_available() and dist.is_initialized():
        if info is not None and info.backend == "nccl":
            dist.barrier(device_ids=[info.local_rank])
        else:
            dist.barrier()


def shutdown():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
