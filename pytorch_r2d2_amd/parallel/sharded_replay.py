"""Replay sharded across data-parallel ranks with globally proportional sampling.

Each rank's HBM replay shard holds the trajectories of its co-located actor group (no frame
bytes ever cross xGMI).  Proportional sampling over the union of shards is two-level:

1. ``all_gather`` the 8 shard totals (one float per rank -- the only collective),
2. each rank keeps its fixed per-rank batch B (static shapes for HIP graphs) and samples
   proportionally *within* its shard; the global sampling probability of sequence i in shard k
   is  P(i) = (p_i / S_k) * (1 / world)  (stratified by shard), so the IS weight uses
   N_global * P(i) with N_global = sum of the shards' valid-sequence counts.

``shard_is_weights`` converts local probabilities into globally consistent IS weights; the
HIP TD kernel accepts them through its ``probs`` input (prob_global = prob_local / world) and
the all-gathered N.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist


def gather_shard_stats(total: torch.Tensor, n_valid: torch.Tensor, world: int, group=None
                       ) -> Tuple[torch.Tensor, torch.Tensor]:
    """total, n_valid: 1-element tensors of this shard -> (totals[world], counts[world])."""
    v = torch.stack([total.reshape(()).float(), n_valid.reshape(()).float()])
    if world <= 1:
        return v[:1].clone(), v[1:].clone()
    out = [torch.zeros_like(v) for _ in range(world)]
    dist.all_gather(out, v, group=group)
    allv = torch.stack(out)
    return allv[:, 0], allv[:, 1]


def shard_is_weights(local_probs: torch.Tensor, world: int, n_global: torch.Tensor,
                     beta: float) -> torch.Tensor:
    p_global = local_probs / world
    w = (n_global * p_global).clamp_min(1e-30) ** (-beta)
    return w / w.max()
