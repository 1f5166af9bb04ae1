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
        # arrival ticket of the fused tree repair (allocated before any graph capture)
        self.tree_ticket = torch.zeros(1, dtype=torch.int32, device=d) if d.type == "cuda" else None
        # prio_tail_kernel: two grid-barrier counters, the arrival ticket, an error word, and the
        # fused sample's tree-ready flag + sampler ticket (r2_prio_tail_sample)
        self.prio_sync = torch.zeros(8, dtype=torch.int32, device=d) if d.type == "cuda" else None
        self.seed = int(cfg.seed) * 0x9E3779B1 + 12345
        self.heads = np.zeros(n_sub, dtype=np.int64)   # per-sub-ring write heads (host mirror)
        self.total_written = 0
        # trajectory ingest (engine/ingest.py, csrc/kernels/ingest.hip): device-side sub-ring
        # write heads, rows counter and malformed-record flag
        self.ihead = torch.zeros(n_sub, dtype=torch.int64, device=d)
        self.rows_total_d = torch.zeros(1, dtype=torch.int64, device=d)
        self.ingest_err = torch.zeros(1, dtype=torch.int32, device=d)

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

    def sample_batch(self, B: int, out_idx: torch.Tensor, out_prob: torch.Tensor,
                     rows: torch.Tensor, Tn: int, states, stream=None, h_f32: bool = False,
                     qreset: Optional[torch.Tensor] = None) -> None:
        """One launch (replay.hip sample_batch_kernel): sample B sequence starts, write the
        time-major row list ``rows[t*B + b]`` (t < Tn) and gather stored states.  ``states``:
        up to 3 ``(hs_cs, offset, h_out (B,H) bf16 -- fp32 with h_f32 --, c_out f32 (B,H))``.
        ``qreset``: the hoisted target torso's frame-queue words, zeroed by the same launch
        (learner_engine.py, learner.hoist)."""
        hs = np.asarray([ptr(s[0]) for s in states] + [0], dtype=np.int64)
        off = np.asarray([int(s[1]) for s in states] + [0], dtype=np.int32)
        h = np.asarray([ptr(s[2]) for s in states] + [0], dtype=np.int64)
        c = np.asarray([ptr(s[3]) for s in states] + [0], dtype=np.int64)
        base = (ptr(self.tree), self.tree_offs.ctypes.data, self.tree_sizes.ctypes.data,
                self.tree_levels, B, self.seed, ptr(self.step), ptr(out_idx), ptr(out_prob), ptr(rows),
                Tn, self.cap_e, self.H, len(states), hs.ctypes.data, off.ctypes.data, h.ctypes.data,
                c.ctypes.data)
        if qreset is not None:
            check(kernels().r2_sample_batch_q(*base, int(h_f32), ptr(qreset), self._ts(stream)),
                  "sample_batch_q")
            return
        fn = kernels().r2_sample_batch_f32h if h_f32 else kernels().r2_sample_batch
        check(fn(*base, self._ts(stream)), "sample_batch")

    def rebuild_tree(self, stream=None) -> None:
        k = kernels()
        check(k.r2_tree_rebuild(ptr(self.tree), self.tree_offs.ctypes.data, self.tree_sizes.ctypes.data,
                                self.tree_levels, self._ts(stream)), "tree_rebuild")

    def update_tree(self, stream=None) -> None:
        k = kernels()
        check(k.r2_tree_update(ptr(self.tree), self.tree_offs.ctypes.data, self.tree_sizes.ctypes.data,
                               self.tree_levels, ptr(self.dirty), ptr(self.dirty_count),
                               self.max_dirty, self._ts(stream)), "tree_update")

    def update_tree_and_end_step(self, end_step: bool = True, stream=None) -> bool:
        """Learner tail: tree repair in two launches (level 0, then level 1 with the small upper
        levels folded in by the last-arriving workgroup, replay.hip tree_update_tail_kernel) and,
        with ``end_step``, the step counter + dirty-list reset in the same launch.  Returns False
        (nothing launched) when the tree shape does not allow the fold."""
        if self.tree_ticket is None:
            if self.tree.device.type != "cuda":
                return False
            self.tree_ticket = torch.zeros(1, dtype=torch.int32, device=self.tree.device)
        rc = kernels().r2_tree_update_fused(
            ptr(self.tree), self.tree_offs.ctypes.data, self.tree_sizes.ctypes.data,
            self.tree_levels, ptr(self.dirty), ptr(self.dirty_count), self.max_dirty,
            ptr(self.tree_ticket), ptr(self.step) if end_step else 0, self._ts(stream))
        if rc == -3:
            return False
        check(rc, "tree_update_fused")
        return True

    def update_tree_and_reset_dirty(self, stream=None) -> bool:
        """The fused tree repair with the dirty-list reset but NOT the step counter (the priority
        tail on a side stream; the counter follows on the main stream, ``step_inc``).  False
        (nothing launched) when the tree shape does not allow the fold."""
        if self.tree_ticket is None:
            if self.tree.device.type != "cuda":
                return False
            self.tree_ticket = torch.zeros(1, dtype=torch.int32, device=self.tree.device)
        rc = kernels().r2_tree_update_fused_reset(
            ptr(self.tree), self.tree_offs.ctypes.data, self.tree_sizes.ctypes.data,
            self.tree_levels, ptr(self.dirty), ptr(self.dirty_count), self.max_dirty,
            ptr(self.tree_ticket), self._ts(stream))
        if rc == -3:
            return False
        check(rc, "tree_update_fused_reset")
        return True

    def prio_tail(self, starts: torch.Tensor, B: int, upd_lo: int, upd_hi: int,
                  end_step: bool = True, stream=None, pack=None) -> bool:
        """The learner's priority tail in ONE launch (replay.hip prio_tail_kernel): sequence
        priorities of the sampled windows, tree repair of every dirty leaf (grid barriers between
        the levels, the upper levels by the last-arriving workgroup) and, with ``end_step``, the
        step counter + dirty-list reset -- bit-identical to refresh_sequences +
        update_tree_and_end_step.  False (nothing launched) when the shape does not allow it."""
        if self.tree.device.type != "cuda":
            return False
        rc = self.cfg.replay
        args = (ptr(starts), B, ptr(self.is_start), ptr(self.priority), ptr(self.tree),
                self.tree_offs.ctypes.data, self.tree_sizes.ctypes.data, self.tree_levels, rc.seq_len,
                upd_lo, upd_hi, self.cap_e, float(rc.eta), ptr(self.dirty), ptr(self.dirty_count),
                self.max_dirty, ptr(self.prio_sync), ptr(self.step) if end_step else 0,
                1 if end_step else 0)
        if pack is not None:
            # + the step's weight repack on extra workgroups (replay.hip r2_prio_tail_pack):
            # ``pack`` = the r2_pack_step arguments between ``step`` and the stream
            if not end_step:
                raise ValueError("prio_tail(pack=...) must end the step")
            r = kernels().r2_prio_tail_pack(*args, *pack, self._ts(stream))
        else:
            r = kernels().r2_prio_tail(*args, self._ts(stream))
        if r in (-3, -4):    # shape, or more workgroups than can be resident at once
            return False
        check(r, "prio_tail")
        return True

    def prio_tail_sample(self, starts: torch.Tensor, B: int, upd_lo: int, upd_hi: int, out_idx,
                         out_prob, rows, Tn: int, states, h_f32: bool, qreset, skip_xcds: int = 0,
                         stream=None) -> bool:
        """prio_tail (ending the step) + the NEXT step's sample_batch in ONE launch (replay.hip
        r2_prio_tail_sample): the sample waits for the repaired tree inside the launch.  Same
        arguments as prio_tail + sample_batch; False (nothing launched) when the shape refuses.
        ``skip_xcds``: keep the launch's workgroups off the first XCDs (the BPTT recurrence's,
        lstm_persist.hip xcd_map 3) -- placement only, same results."""
        if self.tree.device.type != "cuda":
            return False
        rc = self.cfg.replay
        hs = np.asarray([ptr(s_[0]) for s_ in states] + [0], dtype=np.int64)
        off = np.asarray([int(s_[1]) for s_ in states] + [0], dtype=np.int32)
        h = np.asarray([ptr(s_[2]) for s_ in states] + [0], dtype=np.int64)
        c = np.asarray([ptr(s_[3]) for s_ in states] + [0], dtype=np.int64)
        r = kernels().r2_prio_tail_sample(
            ptr(starts), B, ptr(self.is_start), ptr(self.priority), ptr(self.tree),
            self.tree_offs.ctypes.data, self.tree_sizes.ctypes.data, self.tree_levels, rc.seq_len,
            upd_lo, upd_hi, self.cap_e, float(rc.eta), ptr(self.dirty), ptr(self.dirty_count),
            self.max_dirty, ptr(self.prio_sync), ptr(self.step), self.seed, ptr(out_idx),
            ptr(out_prob), ptr(rows), Tn, self.H, len(states), hs.ctypes.data, off.ctypes.data,
            h.ctypes.data, c.ctypes.data, int(h_f32), ptr(qreset), int(skip_xcds), self._ts(stream))
        if r in (-3, -4):
            return False
        check(r, "prio_tail_sample")
        return True

    def reset_dirty(self, stream=None) -> None:
        check(kernels().r2_step_end(0, ptr(self.dirty_count), self._ts(stream)), "reset_dirty")

    def step_inc(self, stream=None) -> None:
        """Step counter + 1 only (the dirty list is reset by the side-stream tree tail)."""
        check(kernels().r2_step_end(ptr(self.step), 0, self._ts(stream)), "step_inc")

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

    # ------------------------------------------------------------------ ingestion (host -> HBM)
    def repair_after_ingest(self, full: bool = False) -> None:
        """Sum-tree repair after ingest launches: the dirty list, or a full rebuild when a record
        was too large for it."""
        if full:
            self.rebuild_tree()
        else:
            self.update_tree()
        self.dirty_count.zero_()

    def ingest_device_record(self, rec: torch.Tensor, head: Optional[np.ndarray], subring: int,
                             repair: bool = True) -> int:
        """Scatter a packed record (``parallel.trajectory.pack_rows``) that already lives in device
        memory (64-byte aligned) into sub-ring ``subring`` (csrc/kernels/ingest.hip).  ``head``:
        the record header on the host if known (only to report the row count)."""
        from ..parallel.trajectory import record_layout
        from .ingest import ingest_args
        n = record_layout(head)[0] if head is not None else 0
        use_dirty = head is not None and min(n, self.cap_e) * 2 <= self.max_dirty
        a = ingest_args(self, ptr(rec), rec.numel(), subring, use_dirty)
        import ctypes
        check(kernels().r2_ingest_record(ctypes.byref(a), ctypes.c_void_p(stream_handle())), "ingest")
        if repair:
            self.repair_after_ingest(full=not use_dirty)
        kept = min(n, self.cap_e)
        self.total_written += kept
        return kept

    @torch.no_grad()
    def ingest_memory(self, mem, subring: Optional[int] = None) -> int:
        """Write a ReplayMemory-schema dict (numpy / tensors, e.g. an actor transport file) as a
        contiguous block into one sub-ring: packed once on the host, one async H2D copy, then the
        device ingest kernel (no host read-back, dirty-list tree repair)."""
        from ..parallel.trajectory import pack_rows
        n = int(mem["state"].shape[0])
        if n == 0:
            return 0
        sub = (self.total_written // max(n, 1)) % self.n_sub if subring is None else subring % self.n_sub
        mem = {k: (v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v)) for k, v in mem.items()}
        if self.obs is not None:
            return self._ingest_obs(mem, sub)
        buf = pack_rows(mem)
        host = torch.from_numpy(buf)
        if self.device.type == "cuda":
            host = host.pin_memory()
        dev = torch.empty(buf.size + 64, dtype=torch.uint8, device=self.device)
        off = (-dev.data_ptr()) % 64
        rec = dev[off: off + buf.size]
        rec.copy_(host, non_blocking=True)
        kept = self.ingest_device_record(rec, buf[:512], sub)
        self._keep_alive = (host, dev)     # until the async copy has been consumed
        return kept

    def _ingest_obs(self, mem, sub: int) -> int:
        """Vector observations (fp32 rows, CartPole): torch scatter path."""
        n = int(mem["state"].shape[0])
        keep = min(n, self.cap_e)
        sl = slice(n - keep, n)
        head = int(self.heads[sub])
        base = sub * self.cap_e
        rows = torch.as_tensor(base + (head + np.arange(keep)) % self.cap_e, device=self.device)
        t = lambda k: torch.as_tensor(np.asarray(mem[k])[sl]).to(self.device)  # noqa: E731
        self.obs[rows] = t("state").reshape(keep, -1).float()
        self.hs_cs[rows] = t("hs_cs").float()
        self.target_hs_cs[rows] = t("target_hs_cs").float()
        self.action[rows] = t("action").reshape(-1).to(torch.uint8)
        self.reward[rows] = t("reward").reshape(-1).float()
        self.done[rows] = (t("done").reshape(-1) > 0).to(torch.uint8)
        self.priority[rows] = t("priority").reshape(-1).float()
        starts = t("is_seq_start").reshape(-1).to(torch.uint8)
        old = self.is_start[rows].to(torch.int32)
        self.n_valid.add_((starts.to(torch.int32) - old).sum().view(1).to(torch.int32))
        self.is_start[rows] = starts
        self.tree[rows] = t("sequence_priority").reshape(-1).float() * starts.float()
        self.heads[sub] = (head + keep) % self.cap_e
        self.total_written += keep
        self.rebuild_tree()
        return keep

    def ingest_file(self, path: str, actor_id: int) -> int:
        """Consume ``memory{actor_id}.pt`` written by a (compat) actor into HBM."""
        import os
        from ..replay.memory import ReplayMemory
        from ..runtime import FileLock
        fpath = os.path.join(path, f"memory{actor_id}.pt")
        if not (os.path.isfile(fpath) and os.path.getsize(fpath) > 0):
            return 0
        lock = FileLock(fpath)
        try:
            if not lock.acquire(blocking=False):
                return 0
            mem = ReplayMemory.read_file(fpath)
            n = self.ingest_memory(mem, subring=actor_id)
            os.remove(fpath)
            return n
        finally:
            lock.release()
            lock.close()

    # ------------------------------------------------------------------ device-side row writes
    @torch.no_grad()
    def clear_rows(self, rows: torch.Tensor) -> None:
        """Rows about to be overwritten stop being sequence starts (leaf -> 0, n_valid--)."""
        was = self.is_start[rows].to(torch.int32)
        self.n_valid.sub_(was.sum().view(1))
        self.is_start.index_fill_(0, rows, 0)      # (index_fill_: no host scalar copy, capturable)
        self.tree.index_fill_(0, rows, 0.0)
        self._append_dirty(rows)

    def _append_dirty(self, rows: torch.Tensor) -> None:
        """Append rows to the dirty list (device-side, no host sync)."""
        n = rows.numel()
        if n == 0:
            return
        pos = self.dirty_count.long() + torch.arange(n, device=self.device)
        ok = pos < self.max_dirty
        self.dirty[pos.clamp_max(self.max_dirty - 1)] = torch.where(ok, rows.to(torch.int32),
                                                                    self.dirty[pos.clamp_max(self.max_dirty - 1)])
        self.dirty_count.add_(n)

    def mark_starts(self, rows: torch.Tensor, n_rows: Optional[torch.Tensor] = None) -> None:
        """Mark sequence starts (rows < 0 are ignored) and set their eta-mixed leaf priority."""
        rc = self.cfg.replay
        k = kernels()
        check(k.r2_mark_starts(ptr(rows), ptr(n_rows), rows.numel(), ptr(self.is_start),
                               ptr(self.priority), ptr(self.tree), rc.seq_len, self.cap_e,
                               float(rc.eta), ptr(self.n_valid), ptr(self.dirty),
                               ptr(self.dirty_count), self.max_dirty, stream_handle()), "mark_starts")

    def flush_tree(self) -> None:
        """Repair the tree for all dirty leaves and reset the dirty list."""
        self.update_tree()
        self.dirty_count.zero_()
