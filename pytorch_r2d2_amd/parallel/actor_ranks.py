"""Actor ranks: GPU actor groups on ranks that own no learner (the split topology).

Reference: N actor processes push experience to ONE learner through pickled files and pull
weights from a Manager dict (``/root/reference/main.py:20-27``, ``replay_memory.py:125-173``,
``learner.py:122-124``, ``actor.py:137-142``).  With ``dist.actor_ranks = A`` of the W ranks (one
process per GPU, torchrun):

* ranks 0 .. L-1 (L = W - A) are data-parallel learner ranks (their replay shards + a
  ``LearnerEngine`` over the learner group); ranks L .. W-1 run ``BatchedActor`` groups only (E
  envs each, the whole GPU for inference and env steps);
* actor rank a feeds learner rank (a - L) % L.  Every round (K env steps) it packs, per env, the
  window of its last K + W - 1 replay rows (W = T + n: the previous window's last W - 1 rows travel
  again, so each sequence's whole window is in exactly ONE record and only the starts whose
  window lies inside the record are kept) with the device pack kernel
  (``csrc/kernels/ingest.hip`` pack_rows_kernel) and sends the fixed-size record with one RCCL
  send; the learner receives it into device memory and scatters it into that actor's E sub-rings
  (env-major ingest);
* weights: every ``publish_rounds`` rounds learner rank 0 broadcasts master + target over the
  {learner 0} + actor-ranks group (``WeightPublisher``: one 2 x 8 MB RCCL broadcast); the actors
  re-pack them between env steps.
Every rank issues the same sequence of point-to-point and collective calls per round, so the
protocol needs no handshake.  Over gloo (CPU tests, ranks sharing a GPU) the device buffers are
staged through host tensors.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..ops._lib import check, kernels, ptr, stream_handle
from .trajectory import ORDER, record_spec

_VP = ctypes.c_void_p


class PackArgs(ctypes.Structure):
    """Mirror of ``struct PackArgs`` (csrc/kernels/ingest.hip); size checked against the .so."""
    _fields_ = [(n, _VP) for n in ("frames", "hs_cs", "ths_cs", "action", "reward", "done",
                                   "priority", "is_start", "leaves", "rec")] + [
        ("off", ctypes.c_longlong * len(ORDER)), ("h0", ctypes.c_longlong)] + [
        (n, ctypes.c_int) for n in ("E", "K", "cap_e", "FB", "H2", "start_from", "start_to", "pad_")]


def split_roles(world: int, actor_ranks: int):
    """(learner ranks, actor ranks, {actor rank: learner rank it feeds})."""
    L = world - int(actor_ranks)
    if actor_ranks < 1 or L < 1:
        raise ValueError(f"actor_ranks={actor_ranks} needs 1 <= actor_ranks < world={world}")
    learners, actors = list(range(L)), list(range(L, world))
    return learners, actors, {a: (a - L) % L for a in actors}


def _is_gloo(group=None) -> bool:
    return dist.is_initialized() and dist.get_backend(group) == "gloo"


def _aligned(nbytes: int, device) -> torch.Tensor:
    buf = torch.zeros(nbytes + 64, dtype=torch.uint8, device=device)
    off = (-buf.data_ptr()) % 64
    return buf[off: off + nbytes]


class TrajectoryPusher:
    """Actor-rank side: pack the E env windows of one round and send them to ``dst``."""

    def __init__(self, replay, K: int, dst: int, group=None):
        rp = replay
        self.rp, self.K, self.dst, self.group = rp, int(K), int(dst), group
        self.W = rp.cfg.replay.seq_len + rp.cfg.replay.n_step
        self.R = self.K + self.W - 1                   # rows per env window
        if self.R + self.K > rp.cap_e:
            raise ValueError(f"actor-rank sub-ring of {rp.cap_e} rows < window {self.R} + round {self.K}")
        self.E = rp.n_sub
        hdr, offs, total = record_spec(self.E * self.R, rp.frame_bytes, 2 * rp.H)
        self.nbytes = total
        self.rec = _aligned(total, rp.device)
        self.rec[: hdr.size].copy_(torch.from_numpy(hdr))
        self.host = torch.empty(total, dtype=torch.uint8, pin_memory=rp.device.type == "cuda") \
            if _is_gloo(group) else None
        if ctypes.sizeof(PackArgs) != kernels().r2_pack_args_bytes():
            raise RuntimeError("PackArgs layout differs from csrc/kernels/ingest.hip")
        a = PackArgs()
        for name, t in (("frames", rp.frames), ("hs_cs", rp.hs_cs), ("ths_cs", rp.target_hs_cs),
                        ("action", rp.action), ("reward", rp.reward), ("done", rp.done),
                        ("priority", rp.priority), ("is_start", rp.is_start), ("leaves", rp.tree),
                        ("rec", self.rec)):
            setattr(a, name, ptr(t))
        for i, o in enumerate(offs):
            a.off[i] = o
        a.E, a.K, a.cap_e, a.FB, a.H2 = self.E, self.R, rp.cap_e, rp.frame_bytes, 2 * rp.H
        a.start_to = self.K
        self.args = a
        self.windows = 0

    def pack(self, window: int) -> torch.Tensor:
        """Window c = ring rows [cK - (W-1), (c+1)K) of every env (the first W-1 rows of window 0
        are before the first step: never starts).  Call after the round's K env steps."""
        a = self.args
        a.h0 = (window * self.K - (self.W - 1)) % self.rp.cap_e
        a.start_from = self.W - 1 if window == 0 else 0
        check(kernels().r2_pack_rows(ctypes.byref(a), _VP(stream_handle())), "pack_rows")
        return self.rec

    def push(self, window: int) -> None:
        rec = self.pack(window)
        if self.host is not None:
            self.host.copy_(rec)
            torch.cuda.current_stream(self.rp.device).synchronize() if self.rp.device.type == "cuda" else None
            dist.send(self.host, self.dst, group=self.group)
        else:
            dist.send(rec, self.dst, group=self.group)
        self.windows += 1


class TrajectoryReceiver:
    """Learner side: one fixed-size record per feeding actor rank per round, scattered env-major
    into sub-rings [i E, (i + 1) E) for the i-th source."""

    def __init__(self, replay, srcs: List[int], E: int, K: int, group=None):
        rp = replay
        self.rp, self.srcs, self.E, self.K, self.group = rp, list(srcs), int(E), int(K), group
        self.W = rp.cfg.replay.seq_len + rp.cfg.replay.n_step
        self.R = self.K + self.W - 1
        if rp.n_sub < self.E * len(self.srcs):
            raise ValueError("the learner replay needs E sub-rings per feeding actor rank")
        _, _, total = record_spec(self.E * self.R, rp.frame_bytes, 2 * rp.H)
        self.nbytes = total
        self.recs = [_aligned(total, rp.device) for _ in self.srcs]
        gloo = _is_gloo(group)
        self.host = [torch.empty(total, dtype=torch.uint8) for _ in self.srcs] if gloo else None
        self.rows = 0
        self.records = 0

    def recv_all(self) -> int:
        from ..engine.ingest import ingest_args
        rp = self.rp
        rows_rec = self.E * self.R
        # the dirty list takes every record's rows; past half of it, rebuild
        budget, used, big = rp.max_dirty // 2, 0, False
        for i, src in enumerate(self.srcs):
            if self.host is not None:
                dist.recv(self.host[i], src, group=self.group)
                self.recs[i].copy_(self.host[i], non_blocking=True)
            else:
                dist.recv(self.recs[i], src, group=self.group)
            need = rows_rec
            use_dirty = not big and used + need <= budget
            big |= not use_dirty
            used += need if use_dirty else 0
            a = ingest_args(rp, ptr(self.recs[i]), self.nbytes, i * self.E, use_dirty,
                            rows_per_sub=self.R)
            check(kernels().r2_ingest_record(ctypes.byref(a), _VP(stream_handle())), "ingest")
            self.rows += rows_rec
            self.records += 1
        rp.repair_after_ingest(full=big)
        rp.total_written += rows_rec * len(self.srcs)
        return rows_rec * len(self.srcs)


def broadcast_weights(pub, engine, version: int, actor_weights=None) -> None:
    """One publication round of ``WeightPublisher`` over the {learner 0} + actor-ranks group:
    learner rank 0 passes its engine, actor ranks their (online, target) ``PackedWeights``."""
    if engine is not None:
        pub.publish(engine.master, engine.target, version)
    else:
        pub.publish(None, None, version)
        on, tg, _ = pub.current()
        actor_weights[0].load_flat(on, version)
        actor_weights[1].load_flat(tg, version)
