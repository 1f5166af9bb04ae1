"""HBM-resident prioritized sequence replay.

Parity target: ``/root/reference/replay_memory.py:58-262`` (ReplayMemory row schema, eta-mixed
sequence priorities, prioritized sequence sampling, stored recurrent state).  The reference keeps
this in host numpy (16 GB for 500k rows), scans all rows per sample and ships ~36 MB H2D per
step.  Here the same row schema lives in device memory sized for 288 GB HBM3E:

    frames        uint8  (cap, C*H*W)      obs stack of the row (state*255, lossless)
    hs_cs         fp32   (cap, 2H)         online LSTM [h | c] stored at acting time
    target_hs_cs  fp32   (cap, 2H)         target LSTM [h | c]
    action        uint8  (cap,)
    reward        fp32   (cap,)            n-step discounted return
    done          uint8  (cap,)
    priority      fp32   (cap,)            per-row (|delta|+eps)^alpha
    is_start      uint8  (cap,)            sequence start marker
    tree          fp32   64-ary sum tree; level 0 == sequence_priority (0 at non-starts)

The ring is split into ``n_subrings`` contiguous sub-rings (one per actor env) so every
episode is contiguous and a sequence wraps inside its own sub-ring.  Sampling, priority
refresh and tree repair are HIP kernels (csrc/kernels/replay.hip); nothing here synchronises
with the host inside a learner step.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from ..config import R2D2Config
from ..ops._lib import check, kernels, ptr, stream_handle

FANOUT = 64


def tree_geometry(cap: int):
    sizes = [cap]
    while sizes[-1] > 1:
        sizes.append((sizes[-1] + FANOUT - 1) // FANOUT)
    if len(sizes) < 2:
        sizes.append(1)
    offs = [0]
    for s in sizes[:-1]:
        offs.append(offs[-1] + s)
    return offs, sizes


class HBMReplay:
    def __init__(self, cfg: R2D2Config, device, capacity: Optional[int] = None,
                 n_subrings: Optional[int] = None, frame_bytes: Optional[int] = None):
        self.cfg = cfg
        rc = cfg.replay
        self.device = torch.device(device)
        cap = capacity or rc.capacity
        n_sub = n_subrings or rc.n_subrings
        cap = cap // n_sub * n_sub
        self.capacity, self.n_sub, self.cap_e = cap, n_sub, cap // n_sub
        e = cfg.env
        if frame_bytes is None:
            frame_bytes = (e.channels_per_frame * e.n_stacks * e.frame_h * e.frame_w
                           if cfg.model.torso == "atari" else 0)
        self.frame_bytes = frame_bytes
        H = cfg.model.hidden
        self.H = H
        d = self.device
        self.frames = torch.zeros((cap, max(frame_bytes, 1)), dtype=torch.uint8, device=d)
        self.obs = None
        if cfg.model.torso != "atari":  # vector observations (CartPole): fp32 rows
            self.obs = torch.zeros((cap, e.obs_dim * e.n_stacks), dtype=torch.float32, device=d)
        self.hs_cs = torch.zeros((cap, 2 * H), dtype=torch.float32, device=d)
        self.target_hs_cs = torch.zeros((cap, 2 * H), dtype=torch.float32, device=d)
        self.action = torch.zeros(cap, dtype=torch.uint8, device=d)
        self.reward = torch.zeros(cap, dtype=torch.float32, device=d)
        self.done = torch.zeros(cap, dtype=torch.uint8, device=d)
        self.priority = torch.zeros(cap, dtype=torch.float32, device=d)
        self.is_start = torch.zeros(cap, dtype=torch.uint8, device=d)
        offs, sizes = tree_geometry(cap)
        self.tree_offs = np.asarray(offs, dtype=np.int64)
        self.tree_sizes = np.asarray(sizes, dtype=np.int64)
        self.tree_levels = len(sizes)
        self.tree = torch.zeros(int(offs[-1] + sizes[-1]), dtype=torch.float32, device=d)
        self.max_dirty = 1 << 16
        self.dirty = torch.zeros(self.max_dirty, dtype=torch.int32, device=d)
        self.dirty_count = torch.zeros(1, dtype=torch.int32, device=d)
        self.n_valid = torch.zeros(1, dtype=torch.int32, device=d)
        self.step = torch.zeros(1, dtype=torch.int64, device=d)
        self.seed = int(cfg.seed) * 0x9E3779B1 + 12345
        self.heads = np.zeros(n_sub, dtype=np.int64)   # per-sub-ring write heads (host mirror)
        self.total_written = 0

    # ------------------------------------------------------------------ properties
    @property
    def sequence_priority(self) -> torch.Tensor:
        return self.tree[: self.capacity]

    def nbytes(self) -> int:
        ts = [self.frames, self.hs_cs, self.target_hs_cs, self.action, self.reward, self.done,
              self.priority, self.is_start, self.tree, self.dirty]
        if self.obs is not None:
            ts.append(self.obs)
        return sum(t.numel() * t.element_size() for t in ts)

    def ring_row(self, start, t):
        start = np.asarray(start, dtype=np.int64)
        base = start - start % self.cap_e
        return base + (start - base + t) % self.cap_e

    @property
    def size(self) -> int:
        return min(self.total_written, self.capacity)

    # ------------------------------------------------------------------ device ops
    def _ts(self, stream=None):
        return stream_handle(stream)

    def sample(self, B: int, out_idx: torch.Tensor, out_prob: torch.Tensor, stream=None) -> None:
        k = kernels()
        check(k.r2_tree_sample(ptr(self.tree), self.tree_offs.ctypes.data, self.tree_sizes.ctypes.data,
                               self.tree_levels, B, self.seed, ptr(self.step), ptr(out_idx),
                               ptr(out_prob), self._ts(stream)), "tree_sample")

    def rebuild_tree(self, stream=None) -> None:
        k = kernels()
        check(k.r2_tree_rebuild(ptr(self.tree), self.tree_offs.ctypes.data, self.tree_sizes.ctypes.data,
                                self.tree_levels, self._ts(stream)), "tree_rebuild")

    def update_tree(self, stream=None) -> None:
        k = kernels()
        check(k.r2_tree_update(ptr(self.tree), self.tree_offs.ctypes.data, self.tree_sizes.ctypes.data,
                               self.tree_levels, ptr(self.dirty), ptr(self.dirty_count),
                               self.max_dirty, self._ts(stream)), "tree_update")

    def refresh_sequences(self, starts: torch.Tensor, B: int, upd_lo: int, upd_hi: int,
                          stream=None) -> None:
        rc = self.cfg.replay
        k = kernels()
        check(k.r2_seqprio_refresh(ptr(starts), B, ptr(self.is_start), ptr(self.priority),
                                   ptr(self.tree), rc.seq_len, upd_lo, upd_hi, self.cap_e,
                                   float(rc.eta), ptr(self.dirty), ptr(self.dirty_count),
                                   self.max_dirty, self._ts(stream)), "seqprio_refresh")

    def step_end(self, stream=None) -> None:
        check(kernels().r2_step_end(ptr(self.step), ptr(self.dirty_count), self._ts(stream)),
              "step_end")

    def total_priority(self) -> float:
        return float(self.tree[int(self.tree_offs[-1])].item())

    # ------------------------------------------------------------------ synthetic fill
    @torch.no_grad()
    def fill_synthetic(self, episode_len: int = 400, seed: int = 0) -> None:
        """Fill every sub-ring with synthetic Atari-shaped episodes (benchmarks / tests).

        Frames are uniform random uint8 (random-data rule: no zero-filled operands), stored
        states ~N(0, 0.1), actions uniform, rewards sparse +-1, episode ends every
        ``episode_len`` rows with the last n rows done=1, priorities uniform(0.1, 1].  Sequence
        starts follow the reference segmentation ``range(ep, end-T, stride) + [end-T]``
        (actor.py:159-167).
        """
        cfg, rc = self.cfg, self.cfg.replay
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        cap, d = self.capacity, self.device
        chunk = 1 << 16
        for a in range(0, cap, chunk):
            b = min(cap, a + chunk)
            if self.frame_bytes > 1:
                self.frames[a:b] = torch.randint(0, 256, (b - a, self.frame_bytes), dtype=torch.uint8,
                                                 device=d, generator=g)
        if self.obs is not None:
            self.obs.normal_(0, 1, generator=g)
        self.hs_cs.normal_(0, 0.1, generator=g)
        self.target_hs_cs.normal_(0, 0.1, generator=g)
        self.action.copy_(torch.randint(0, self.cfg.model.n_actions, (cap,), device=d,
                                        generator=g).to(torch.uint8))
        r = torch.rand(cap, device=d, generator=g)
        self.reward.copy_(torch.where(r < 0.02, 1.0, torch.where(r > 0.98, -1.0, 0.0)))
        self.priority.copy_(torch.rand(cap, device=d, generator=g) * 0.9 + 0.1)
        T, n, stride = rc.seq_len, rc.n_step, rc.overlap
        L = max(episode_len, T + n)
        pos = torch.arange(cap, device=d) % self.cap_e
        ep_pos = pos % L
        ep_len = torch.full_like(pos, L)
        tail = (self.cap_e // L) * L
        last_partial = pos >= tail
        ep_len = torch.where(last_partial, self.cap_e - tail, ep_len)
        self.done.copy_((ep_pos >= ep_len - n).to(torch.uint8))
        starts = ((ep_pos % stride == 0) & (ep_pos < ep_len - T - n + 1)) | (ep_pos == ep_len - T - n)
        starts &= ep_len >= T + n
        self.is_start.copy_(starts.to(torch.uint8))
        self.n_valid.fill_(int(starts.sum().item()))
        # eta-mix over the T rows of each start (vectorised with ring wrap inside sub-ring)
        idx = torch.nonzero(starts).squeeze(1)
        tt = torch.arange(T, device=d)
        base = idx - idx % self.cap_e
        rows = base[:, None] + (idx[:, None] - base[:, None] + tt[None, :]) % self.cap_e
        p = self.priority[rows]
        seqp = rc.eta * p.max(1).values + (1 - rc.eta) * p.mean(1)
        self.tree.zero_()
        self.tree[idx] = seqp
        self.total_written = cap
        self.heads[:] = 0
        self.rebuild_tree()
        torch.cuda.synchronize(d) if d.type == "cuda" else None
