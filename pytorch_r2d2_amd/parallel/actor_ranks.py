"""Actor ranks: GPU actor groups on ranks that own no learner (the split topology).

Reference: N actor processes push experience to ONE learner through pickled files and pull
weights from a Manager dict, never waiting for each other (``/root/reference/main.py:20-27``,
``actor.py:64-66``, ``learner.py:53-66``, ``replay_memory.py:125-173``, ``learner.py:122-124``,
``actor.py:137-142``).  With ``dist.actor_ranks = A`` of the W ranks (one process per GPU,
torchrun):

* ranks 0 .. L-1 (L = W - A <= A) are data-parallel learner ranks (their replay shards + a
  ``LearnerEngine`` over the learner group); ranks L .. W-1 run ``BatchedActor`` groups only (E
  envs each, the whole GPU for inference and env steps);
* actor rank a feeds learner rank (a - L) % L through an asynchronous link
  (``parallel/channel.py``): every K env steps it packs, per env, the K newest FINAL rows (the
  rows K + n .. n + 1 steps old: a row's n-step return, done flag and priority are final n steps
  after it is written) with the device pack kernel (``csrc/kernels/ingest.hip``) and sends them;
  each row travels exactly once.  A sequence start travels with the last row of its window
  (start column lagged by W - 1 = T + n - 1 rows), so the learner's sub-ring -- one contiguous
  stream per env -- only ever holds starts whose whole window it has received;
* the learner polls its links between steps and ingests whatever has arrived (env-major
  device ingest); it never waits for a particular actor, and an actor blocks only when all of
  its ``dist.push_slots`` records are still untaken;
* weights: every ``dist.publish_steps`` learner steps learner rank 0 sends master + target to
  each actor rank whose previous snapshot has been taken (one 2 x 8 MB message, RCCL); actor
  ranks take snapshots between rounds.
Over gloo (CPU tests, ranks sharing a GPU) the device buffers are staged through host tensors.
"""
from __future__ import annotations

import ctypes
import time
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
        (n, ctypes.c_int) for n in ("E", "K", "cap_e", "FB", "H2", "start_from", "start_to", "lag")]


def split_roles(world: int, actor_ranks: int):
    """(learner ranks, actor ranks, {actor rank: learner rank it feeds}).  Every learner needs at
    least one feeding actor rank (a learner without one never fills its replay, and the data-
    parallel learners start only when every shard holds a batch)."""
    L = world - int(actor_ranks)
    if actor_ranks < 1 or L < 1:
        raise ValueError(f"actor_ranks={actor_ranks} needs 1 <= actor_ranks < world={world}")
    if actor_ranks < L:
        raise ValueError(f"actor_ranks={actor_ranks} < learner ranks {L}: every learner rank needs "
                         f"an actor rank feeding it")
    learners, actors = list(range(L)), list(range(L, world))
    return learners, actors, {a: (a - L) % L for a in actors}


def _is_gloo(group=None) -> bool:
    return dist.is_initialized() and dist.get_backend(group) == "gloo"


def record_link(actor_rank: int) -> str:
    return f"r2d2/rec/{actor_rank}"


def weight_link(actor_rank: int) -> str:
    return f"r2d2/w/{actor_rank}"


class TrajectoryPusher:
    """Actor-rank side: every K env steps pack the E env blocks of K final rows and send them to
    learner rank ``dst`` over an asynchronous link with ``slots`` record buffers."""

    def __init__(self, replay, K: int, dst: int, slots: int = 4, group=None, link=True):
        rp = replay
        self.rp, self.K, self.dst, self.group = rp, int(K), int(dst), group
        self.n = rp.cfg.replay.n_step
        self.W = rp.cfg.replay.seq_len + self.n
        self.lag = self.W - 1
        if self.K + self.n + self.W > rp.cap_e:
            raise ValueError(f"actor-rank sub-ring of {rp.cap_e} rows < round {self.K} + n {self.n} "
                             f"+ window {self.W}")
        self.E = rp.n_sub
        hdr, offs, total = record_spec(self.E * self.K, rp.frame_bytes, 2 * rp.H)
        self.nbytes = total
        self.hdr = torch.from_numpy(hdr)
        if ctypes.sizeof(PackArgs) != kernels().r2_pack_args_bytes():
            raise RuntimeError("PackArgs layout differs from csrc/kernels/ingest.hip")
        a = PackArgs()
        for name, t in (("frames", rp.frames), ("hs_cs", rp.hs_cs), ("ths_cs", rp.target_hs_cs),
                        ("action", rp.action), ("reward", rp.reward), ("done", rp.done),
                        ("priority", rp.priority), ("is_start", rp.is_start), ("leaves", rp.tree)):
            setattr(a, name, ptr(t))
        for i, o in enumerate(offs):
            a.off[i] = o
        a.E, a.K, a.cap_e, a.FB, a.H2 = self.E, self.K, rp.cap_e, rp.frame_bytes, 2 * rp.H
        a.start_to, a.lag = self.K, self.lag
        self.args = a
        self.link = None
        if link:
            from .channel import LinkSender
            self.link = LinkSender(record_link(dist.get_rank()), self.dst, total, slots, rp.device,
                                   data_group=group, host_stage=_is_gloo(group))
            for b in self.link.bufs:
                b[: hdr.size].copy_(self.hdr)
        self.windows = 0

    def pack(self, window: int, rec: torch.Tensor) -> torch.Tensor:
        """Block c = stream rows [cK - n, (c+1)K - n) of every env (all final after the round's K
        env steps), start column of stream rows [cK - n - (W-1), ...) -- stream rows < 0 carry no
        starts.  Call after the round's K env steps."""
        a = self.args
        a.rec = ptr(rec)
        a.h0 = (window * self.K - self.n) % self.rp.cap_e
        a.start_from = max(0, self.lag + self.n - window * self.K)
        check(kernels().r2_pack_rows(ctypes.byref(a), _VP(stream_handle())), "pack_rows")
        return rec

    def push(self, window: int) -> None:
        rec = self.link.acquire()
        self.pack(window, rec)
        self.link.send()
        self.windows += 1

    def finish(self) -> None:
        self.link.flush()
        self.link.close()


class TrajectoryReceiver:
    """Learner side: the links of the actor ranks ``srcs``; ``poll()`` ingests every record that
    has arrived, env-major into sub-rings [i E, (i + 1) E) for the i-th source."""

    def __init__(self, replay, srcs: List[int], E: int, K: int, group=None):
        from .channel import LinkReceiver
        rp = replay
        self.rp, self.srcs, self.E, self.K, self.group = rp, list(srcs), int(E), int(K), group
        self.n = rp.cfg.replay.n_step
        self.lag = rp.cfg.replay.seq_len + self.n - 1
        if rp.n_sub < self.E * len(self.srcs):
            raise ValueError("the learner replay needs E sub-rings per feeding actor rank")
        _, _, total = record_spec(self.E * self.K, rp.frame_bytes, 2 * rp.H)
        self.nbytes = total
        self.rows = 0
        self.records = 0
        self._budget = 0
        self._big = False
        self.link = LinkReceiver([record_link(a) for a in self.srcs], self.srcs, total, rp.device,
                                 self._ingest, data_group=group, host_stage=_is_gloo(group))

    def _ingest(self, i: int, rec: torch.Tensor) -> None:
        from ..engine.ingest import ingest_args
        rp = self.rp
        need = 2 * self.E * self.K          # a data row and a start row per record row
        use_dirty = not self._big and self._budget + need <= rp.max_dirty // 2
        self._big |= not use_dirty
        self._budget += need if use_dirty else 0
        a = ingest_args(rp, ptr(rec), self.nbytes, i * self.E, use_dirty, rows_per_sub=self.K,
                        start_lag=self.lag)
        check(kernels().r2_ingest_record(ctypes.byref(a), _VP(stream_handle())), "ingest")
        self.rows += self.E * self.K
        self.records += 1
        rp.total_written += self.E * self.K

    def poll(self, **kw) -> int:
        self._budget, self._big = 0, False
        got = self.link.poll(**kw)
        if got:
            self.rp.repair_after_ingest(full=self._big)
        return got

    def drain(self, rounds: int) -> None:
        """Block until every source has delivered ``rounds`` records (end of a run)."""
        while any(r < rounds for r in self.link.received):
            if self.poll() == 0:
                time.sleep(0.0005)


class WeightLinks:
    """Learner rank 0 -> actor ranks: master + target snapshots ([online | target] fp32) over one
    single-slot link per actor rank, published only to actors that took the previous one."""

    def __init__(self, numel: int, device, actors: List[int], src: int, role: str, group=None):
        from .channel import LinkReceiver, LinkSender
        self.numel = int(numel)
        nbytes = 2 * self.numel * 4
        stage = _is_gloo(group)
        self.published = 0
        self.senders, self.receiver = [], None
        if role == "learner":
            self.senders = [LinkSender(weight_link(a), a, nbytes, 1, device, data_group=group,
                                       tag=1, host_stage=stage) for a in actors]
        else:
            self.taken = 0
            self.receiver = LinkReceiver([weight_link(dist.get_rank())], [src], nbytes, device,
                                         self._load, data_group=group, tag=1, host_stage=stage)
            self.targets = None

    def publish(self, master: torch.Tensor, target: torch.Tensor) -> int:
        """Learner 0: send to every actor rank whose previous snapshot was taken (non-blocking
        apart from one store round trip per actor rank).  Returns how many were sent."""
        sent = 0
        for tx in self.senders:
            if tx.in_flight() == 0:
                buf = tx.acquire().view(torch.float32)
                buf[: self.numel].copy_(master.reshape(-1)[: self.numel])
                buf[self.numel:].copy_(target.reshape(-1)[: self.numel])
                tx.send()
                sent += 1
        self.published += 1 if sent else 0
        return sent

    def close(self) -> None:
        for tx in self.senders:
            tx.flush()
            tx.close()

    # actor side
    def attach(self, online, target) -> None:
        self.targets = (online, target)

    def _load(self, i: int, buf: torch.Tensor) -> None:
        f = buf.view(torch.float32)
        self.taken += 1
        self.targets[0].load_flat(f[: self.numel], self.taken)
        self.targets[1].load_flat(f[self.numel:], self.taken)

    def poll(self) -> int:
        return self.receiver.poll()

    def wait_closed(self) -> None:
        self.receiver.wait_closed()
