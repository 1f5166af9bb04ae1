"""Learner -> actor weight publication.

Reference: the learner pickles ``deepcopy(net).cpu().state_dict()`` for net and target into a
``multiprocessing.Manager`` dict every 100 steps (learner.py:122-124) and actors unpickle them
every 5 episodes under a bare ``except`` (actor.py:137-142); net and target are read without a
version, so an actor can mix weights of different steps.

``WeightPublisher`` (device side, RCCL): the learner rank owns the flat fp32 master buffers of
the online and target nets.  ``publish()`` copies both into a double-buffered, versioned slot
pair and ``dist.broadcast``s the slot (one 2 x 8 MB message) from the learner rank to every rank
in the group; receivers get a consistent (online, target, version) triple and swap it in
atomically.  When actor and learner share a GPU the actor simply reads the engine's packed
buffers (zero copy; ``actor_batched.engine_weights``).

``SharedDictWeights`` keeps the reference's Manager-dict contract (keys ``net_state``,
``target_net_state``) plus a ``version`` key, for the compat process topology.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist


class WeightPublisher:
    def __init__(self, numel: int, device, src_rank: int = 0, group=None):
        self.numel = numel
        self.src = src_rank
        self.group = group
        d = torch.device(device)
        # slot layout: [online (numel) | target (numel) | version (1)]
        self.slots = [torch.zeros(2 * numel + 1, dtype=torch.float32, device=d) for _ in range(2)]
        self.front = 0
        self.version = -1

    def publish(self, online: Optional[torch.Tensor], target: Optional[torch.Tensor],
                version: int) -> None:
        """Collective: every rank of the group calls it; the src rank provides the weights."""
        back = self.slots[1 - self.front]
        rank = dist.get_rank() if dist.is_initialized() else 0
        if rank == self.src:
            back[: self.numel].copy_(online.reshape(-1)[: self.numel])
            back[self.numel: 2 * self.numel].copy_(target.reshape(-1)[: self.numel])
            back[-1] = float(version)
        if dist.is_initialized() and dist.get_world_size(self.group) > 1:
            dist.broadcast(back, src=self.src, group=self.group)
        self.front = 1 - self.front
        # every rank of the group calls publish with the same host-side version counter: no
        # device read-back (the version word in the slot is for consumers reading it on device)
        self.version = int(version)

    def current(self) -> Tuple[torch.Tensor, torch.Tensor, int]:
        s = self.slots[self.front]
        return s[: self.numel], s[self.numel: 2 * self.numel], self.version


class SharedDictWeights:
    """Reference-compatible Manager-dict transport with a version stamp."""

    def __init__(self, shared_dict):
        self.d = shared_dict

    def publish(self, online_sd, target_sd, version: int) -> None:
        self.d["net_state"] = {k: v.detach().cpu() for k, v in online_sd.items()}
        self.d["target_net_state"] = {k: v.detach().cpu() for k, v in target_sd.items()}
        self.d["version"] = version

    def fetch(self):
        return self.d["net_state"], self.d["target_net_state"], self.d.get("version", -1)


class ShmWeightsWriter:
    """Learner side of the native CPU-actor weight transport: the flat fp32 master buffers of the
    online and target nets go device -> pinned host (async, on the learner's stream) -> a
    shared-memory seqlock slot (``runtime.ShmSlot``) that every CPU actor process reads.  No
    learner-stream synchronisation: ``publish`` enqueues the copy and records an event; ``poll``
    writes the slot once that event has completed (called from the learner loop)."""

    def __init__(self, name: str, numel: int, device):
        from ..runtime import ShmSlot
        self.numel = int(numel)
        self.slot = ShmSlot(name, 2 * self.numel * 4, create=True)
        pin = torch.device(device).type == "cuda"
        self.host = torch.zeros(2 * self.numel, dtype=torch.float32, pin_memory=pin)
        self.event = torch.cuda.Event() if pin else None
        self.pending: Optional[int] = None
        self.version = -1

    def publish(self, online: torch.Tensor, target: torch.Tensor, version: int) -> None:
        if self.pending is not None:
            self.poll(wait=True)
        self.host[: self.numel].copy_(online.reshape(-1)[: self.numel], non_blocking=True)
        self.host[self.numel:].copy_(target.reshape(-1)[: self.numel], non_blocking=True)
        if self.event is not None:
            self.event.record()
        self.pending = int(version)
        self.poll()

    def poll(self, wait: bool = False) -> bool:
        if self.pending is None:
            return False
        if self.event is not None and not self.event.query():
            if not wait:
                return False
            self.event.synchronize()
        self.slot.write(self.host.numpy(), self.pending)
        self.version, self.pending = self.pending, None
        return True

    def close(self):
        self.slot.close(unlink=True)


class ShmWeightsReader:
    """CPU actor side: ``fetch(have)`` returns (online_sd, target_sd, version) when a version newer
    than ``have`` is published, else None.  Reads are seqlock-consistent (never torn)."""

    def __init__(self, name: str, cfg=None):
        from ..config import get_config
        from ..engine.layout import ParamLayout
        from ..runtime import ShmSlot
        cfg = cfg or get_config("reference")
        self.layout = ParamLayout(cfg.model, cfg.env)
        self.numel = int(self.layout.padded)
        self.slot = ShmSlot(name, 2 * self.numel * 4, create=False)
        self.buf = np.zeros(2 * self.numel, dtype=np.float32)

    def fetch(self, have: int = -1):
        v = self.slot.read(self.buf, have)
        if v is None:
            return None
        t = torch.from_numpy(self.buf.copy())
        return (self.layout.state_dict(t[: self.numel]), self.layout.state_dict(t[self.numel:]), v)
