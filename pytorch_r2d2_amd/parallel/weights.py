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
        self.version = int(back[-1].item())

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
