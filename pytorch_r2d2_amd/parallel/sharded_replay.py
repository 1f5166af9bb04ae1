"""Replay sharded across data-parallel ranks with globally proportional prioritized sampling.

Reference: one replay, sequences sampled proportionally to their priority
(``/root/reference/replay_memory.py:224-232``: WeightedRandomSampler over sequence_priority).
Here every DP rank's HBM replay shard holds the trajectories of its co-located actor group (no
frame bytes ever cross xGMI), and every rank trains on a fixed-size local batch B (static shapes:
the step is a HIP graph).  Sampling is two-level:

1. each rank draws its B sequences proportionally to priority WITHIN its shard:
   q_k(i) = p_i / S_k (stratified), i.e. shard k contributes B of the W*B global samples;
2. right after sampling, ONE all-gather of 3 floats per rank -- (S_k, N_k, min_b q_k(b)) -- gives
   every rank the global total S = sum S_k, the global sequence count N = sum N_k and the batch
   extremes;
3. sample b of rank k gets the loss weight

       w_b = (W S_k / S) * (N * P(b))^-beta / max_global,      P(b) = p_b / S = q_k(b) * S_k / S

   The first factor is the importance ratio between the global prioritized distribution P and
   the per-shard sampling distribution q_k / W, so the expected weighted gradient equals that of a
   single merged replay sampled proportionally to priority; the second is the usual PER IS
   correction with the global N (replay_memory.py has no IS weights: beta = 0 reduces w_b to the
   shard ratio alone); ``max_global`` (the largest weight of the global batch, computable from the
   gathered minima) keeps w <= 1 exactly as the single-replay normalisation does.

The device side is ``td.hip`` (``TdArgs.dp``: {W S_k/S, S_k/S, N, max_global}); these torch
functions produce those four numbers (graph-capturable tensor ops, no host reads) and are the
CPU reference the tests check the kernels against.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def local_stats(total: torch.Tensor, n_valid: torch.Tensor, probs: torch.Tensor,
                out: torch.Tensor = None) -> torch.Tensor:
    """(3,) fp32 [S_k, N_k, min_b q_k(b)] of this shard (device tensors in, no host sync)."""
    v = torch.stack([total.reshape(()).float(), n_valid.reshape(()).float(),
                     probs.min().reshape(()).float()])
    if out is not None:
        out.copy_(v)
        return out
    return v


def gather_stats(local: torch.Tensor, world: int, group=None, out: torch.Tensor = None
                 ) -> torch.Tensor:
    """(world, 3) all-gathered shard stats (a 12-byte message per rank)."""
    if out is None:
        out = torch.empty(world * 3, dtype=local.dtype, device=local.device)
    if world <= 1:
        out.copy_(local.reshape(-1))
    else:
        dist.all_gather_into_tensor(out, local.reshape(-1), group=group)
    return out.view(world, 3)


def global_is_params(stats: torch.Tensor, rank: int, beta: float,
                     out: torch.Tensor = None) -> torch.Tensor:
    """(4,) [W S_k/S, S_k/S, N, max_global] for rank ``rank`` from the gathered (W, 3) stats."""
    W = stats.shape[0]
    S_k = stats[:, 0]
    S = S_k.sum().clamp_min(1e-30)
    N = stats[:, 1].sum()
    scale = S_k / S
    factor = W * scale
    if beta > 0:
        wmax = factor * (N * stats[:, 2] * scale).clamp_min(1e-30) ** (-beta)
    else:
        wmax = factor
    v = torch.stack([factor[rank], scale[rank], N, wmax.max()])
    if out is not None:
        out.copy_(v)
        return out
    return v


def dp_is_weights(probs: torch.Tensor, params: torch.Tensor, beta: float) -> torch.Tensor:
    """Torch reference of the TD kernel's data-parallel weights (td.hip ``is_weight``)."""
    w = (params[2] * probs * params[1]).clamp_min(1e-30) ** (-beta) if beta > 0 else torch.ones_like(probs)
    return params[0] * w / params[3]


def single_replay_is_weights(p: torch.Tensor, n: float, beta: float) -> torch.Tensor:
    """The single-replay formula w = (N P)^-beta / max (replay over the merged shards)."""
    w = (n * p).clamp_min(1e-30) ** (-beta)
    return w / w.max()
