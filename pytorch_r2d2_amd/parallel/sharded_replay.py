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


def gather_stats(local: torch.Tensor, world: int, group=None, out: torch.Tensor = None,
                 force: bool = False) -> torch.Tensor:
    """(world, 3) all-gathered shard stats (a 12-byte message per rank).  ``force``: run the
    collective at world 1 too (dist.force_dp rehearsal)."""
    if out is None:
        out = torch.empty(world * 3, dtype=local.dtype, device=local.device)
    if world <= 1 and not (force and group is not None):
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


# ---------------------------------------------------------------- variance of the two-level scheme
# Why not per-shard counts drawn by multinomial?  Those would give every step the
# exact distribution of one merged replay, but a rank's batch size would change every step: the
# graphed step needs a static B, and a shard asked for more than B sequences cannot serve them.
# The shard-ratio weights keep B fixed and stay unbiased (the chi-square test pins that); what they
# cost is variance.  For a per-sequence quantity f with within-shard variance V_k and shard means
# mu_k (mu the global mean, s_k = S_k / S):
#
#     Var(local + ratio)  = (1/B) sum_k s_k^2 V_k
#     Var(merged replay)  = 1/(W B) [sum_k s_k V_k + sum_k s_k (mu_k - mu)^2]
#
# With equal within-shard variances the ratio is at most W sum_k s_k^2 (``imbalance_factor``): 1
# for balanced shards, 1 + W sum_k (s_k - 1/W)^2 in general; the between-shard term, which local
# sampling removes (it is stratified over shards), only lowers it.  Co-located actor groups feed
# the shards symmetrically, so s_k ~ 1/W: e.g. +-10 % shard totals at W = 8 cost ~1 % variance.
# ``mc_estimator_variance`` measures all of this (tests/test_sharded_sampling_cpu.py,
# tools/dp_sampling_variance.py -> profiles/r03_dp_sampling_variance.txt).
def imbalance_factor(stats: torch.Tensor) -> torch.Tensor:
    """W * sum_k (S_k / S)^2 from the gathered (W, 3) shard stats (>= 1; 1 = balanced)."""
    s = stats[:, 0] / stats[:, 0].sum().clamp_min(1e-30)
    return stats.shape[0] * (s * s).sum()


def mc_estimator_variance(priorities, values, B: int, trials: int = 4000, seed: int = 0):
    """Monte-Carlo variance of three estimators of E_P[f] (P proportional to priority over the
    union of the shards): ``merged`` (W*B draws from the merged replay), ``multinomial`` (shard
    counts ~ Multinomial(W*B, s), then within-shard draws) and ``local_ratio`` (B draws per shard
    with the shard-ratio weight W s_k -- what the engine does).  priorities / values: lists of
    per-shard numpy arrays.  Returns {name: (mean, variance)} and the true mean."""
    import numpy as np
    g = np.random.default_rng(seed)
    W = len(priorities)
    S = np.asarray([p.sum() for p in priorities])
    s = S / S.sum()
    allp = np.concatenate(priorities) / S.sum()
    allf = np.concatenate(values)
    mu = float((allp * allf).sum())
    q = [p / p.sum() for p in priorities]
    est = {"merged": [], "multinomial": [], "local_ratio": []}
    for _ in range(trials):
        est["merged"].append(allf[g.choice(len(allf), W * B, p=allp)].mean())
        c = g.multinomial(W * B, s)
        est["multinomial"].append(np.concatenate(
            [values[k][g.choice(len(q[k]), c[k], p=q[k])] for k in range(W)]).mean())
        est["local_ratio"].append(sum(W * s[k] * values[k][g.choice(len(q[k]), B, p=q[k])].sum()
                                      for k in range(W)) / (W * B))
    return {k: (float(np.mean(v)), float(np.var(v))) for k, v in est.items()}, mu
