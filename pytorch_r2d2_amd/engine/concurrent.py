"""Concurrent actor group + learner on one MI355X (Ape-X decoupling without a host round trip).

Reference: actors and the learner are separate processes running at the same time
(``/root/reference/main.py:20-33``); the learner publishes weights every 100 steps
(``learner.py:109-110``) and actors pull them every 5 episodes (``actor.py:134-135``).  On the
native path both roles live in one process per GPU and run SIMULTANEOUSLY on disjoint CU sets:

* the two roles get their own streams, either sharing the whole chip (the default: the actor's
  short kernels fill CUs the learner leaves idle, e.g. the 64 outside the persistent LSTM
  forward's 192, and never wait on the learner, so a learner workgroup that finds its CU taken
  waits at most for one actor workgroup) or CU-masked (``parallel/placement.py``: ``k`` CUs of
  every XCD for the actor, the other ``32 - k`` for the learner, whose persistent kernels are
  placed for its own per-XCD CU counts);
* the host issues *rounds*: ``M`` actor env steps (graph replays) on the actor stream and one
  learner step on the learner stream.  Actor round ``r`` waits for learner step ``r - 1``; learner
  step ``r`` waits for actor round ``r - 1``.  Each role therefore overlaps the other's next
  round, with no host synchronisation;
* **replay consistency** -- the learner reads the sequence-start flags / sum tree while the actor
  writes rows, so the actor never touches them (``actor.hip`` deferred mode): start marks and
  clears go to a pending list (two lists, round parity) that the learner's stream applies in front
  of its next step (``replay.hip`` apply_pending_kernel + dirty-list tree repair).  Rows are
  invalidated ``lookahead >= M`` steps ahead of the write head, so a row written in round ``r`` had
  its starts cleared in a round ``<= r - 1``, applied before learner step ``r`` sampled; learner step
  ``r - 1`` (which may still have sampled them) finished before actor round ``r`` started;
* **weights** -- the actor reads its OWN packed copy.  Every ``publish_interval`` learner steps the
  learner's stream copies master + target into a staging slot behind its step, and the actor's
  stream re-packs that slot at the start of its next round (after the event wait), so the actor
  never sees a half-updated optimizer step and weights change only between actor steps.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from ..ops._lib import check, kernels, ptr, stream_handle


class ConcurrentDriver:
    def __init__(self, engine, actor, steps_per_round: int = 2, publish_interval: Optional[int] = None,
                 lookahead: Optional[int] = None, actor_stream=None, learner_stream=None,
                 capture: bool = True, learner_priority: int = 0):
        from ..actor_batched import PackedWeights
        self.eng, self.actor = engine, actor
        self.rp = rp = actor.replay
        if engine.replay is not rp:
            raise ValueError("actor and learner must share one HBM replay")
        self.M = M = int(steps_per_round)
        self.D = D = int(lookahead) if lookahead else M + 2
        if D < M:
            raise ValueError("lookahead must be >= steps_per_round")
        self.P = int(publish_interval or engine.cfg.learner.publish_interval)
        dev = rp.device
        E, n, W = actor.E, actor.n, actor.T + actor.n
        # per round: M steps x E envs x (1 lookahead clear + up to n + 2 marks), one wrap step's
        # W - 1 clears per env
        self.cap = M * E * (n + 3) + E * W
        self.pend = [torch.zeros(self.cap, dtype=torch.int32, device=dev) for _ in range(2)]
        self.cnt = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in range(2)]
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        # the actor's own weights, re-packed from a staging slot the learner fills
        L = actor.layout
        self.stage_on = engine.master.detach().clone()
        self.stage_tg = engine.target.detach().clone()
        self.w_on, self.w_tg = PackedWeights(L, dev), PackedWeights(L, dev)
        self.w_on.load_flat(self.stage_on, 0)
        self.w_tg.load_flat(self.stage_tg, 0)
        self.version = 0
        self._repack = False
        self.s_act = actor_stream if actor_stream is not None else torch.cuda.Stream(device=dev)
        # shared chip (no CU masks): ``learner_priority`` -1 puts the learner's stream on a
        # high-priority queue, so its workgroups win free CUs over the actor's
        self.s_learn = learner_stream if learner_stream is not None else \
            torch.cuda.Stream(device=dev, priority=int(learner_priority))
        self.ev_act = [torch.cuda.Event(), torch.cuda.Event()]
        self.ev_learn = torch.cuda.Event()
        self.rounds = 0
        self.learner_steps = 0
        self.heads = []           # actor write head at the start of every round (tests)
        self.on_learner_step = None   # optional callback(step_idx) on the learner stream
        actor.set_weights(self.w_on, self.w_tg)
        actor.enable_deferred(self.pend, self.cnt, self.cap, D)
        torch.cuda.synchronize(dev)
        # serial switch-over: the D rows ahead of every env's write head stop being starts now
        rows = (torch.arange(E, device=dev, dtype=torch.int64)[:, None] * rp.cap_e
                + (actor.head + torch.arange(D, device=dev)[None, :]) % rp.cap_e).reshape(-1)
        rp.clear_rows(rows)
        rp.flush_tree()
        # one eager deferred step (first launch of every actor kernel outside capture), applied
        actor.step(parity=0)
        self._apply(0)
        torch.cuda.synchronize(dev)
        self.apply_graphs = None
        if capture and dev.type == "cuda":
            with torch.cuda.stream(self.s_act):
                actor.capture(warmup=0)
            torch.cuda.synchronize(dev)
            graphs, pool = [], None
            side = torch.cuda.Stream(device=dev)
            for p in (0, 1):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool, stream=side):
                    self._apply(p)
                pool = g.pool()
                graphs.append(g)
            self.apply_graphs = graphs
            torch.cuda.synchronize(dev)

    # ------------------------------------------------------------------ pieces
    def _apply(self, p: int) -> None:
        """Learner stream: apply pending list ``p``, repair the tree, reset both counts."""
        rp, rc = self.rp, self.eng.cfg.replay
        check(kernels().r2_apply_pending(ptr(self.pend[p]), ptr(self.cnt[p]), self.cap,
                                         ptr(rp.is_start), ptr(rp.priority), ptr(rp.tree),
                                         rc.seq_len, rp.cap_e, float(rc.eta), ptr(rp.n_valid),
                                         ptr(rp.dirty), ptr(rp.dirty_count), rp.max_dirty,
                                         ptr(self.err), stream_handle()), "apply_pending")
        rp.update_tree()
        rp.dirty_count.zero_()
        self.cnt[p].zero_()

    def round(self) -> None:
        r = self.rounds
        p = r & 1
        self.heads.append(self.actor.head)
        with torch.cuda.stream(self.s_act):
            if r > 0:
                self.s_act.wait_event(self.ev_learn)
            if self._repack:
                self.w_on.load_flat(self.stage_on, self.version)
                self.w_tg.load_flat(self.stage_tg, self.version)
                self._repack = False
            for _ in range(self.M):
                self.actor.step(parity=p)
            self.ev_act[p].record(self.s_act)
        with torch.cuda.stream(self.s_learn):
            if r > 0:
                self.s_learn.wait_event(self.ev_act[1 - p])
                self._replay_apply(1 - p)
            self.eng.step()
            if self.on_learner_step is not None:
                self.on_learner_step(self.learner_steps)
            self.learner_steps += 1
            if self.learner_steps % self.P == 0:
                self.stage_on.copy_(self.eng.master)
                self.stage_tg.copy_(self.eng.target)
                self.version += 1
                self._repack = True
            self.ev_learn.record(self.s_learn)
        self.rounds += 1

    def _replay_apply(self, p: int) -> None:
        if self.apply_graphs is not None:
            self.apply_graphs[p].replay()
        else:
            self._apply(p)

    def finish(self) -> None:
        """Apply the last round's pending edits and wait for both streams."""
        if self.rounds > 0:
            p = (self.rounds - 1) & 1
            with torch.cuda.stream(self.s_learn):
                self.s_learn.wait_event(self.ev_act[p])
                self._replay_apply(p)
            if self._repack:   # the actor picks up the last publication
                with torch.cuda.stream(self.s_act):
                    self.s_act.wait_event(self.ev_learn)
                    self.w_on.load_flat(self.stage_on, self.version)
                    self.w_tg.load_flat(self.stage_tg, self.version)
                self._repack = False
        torch.cuda.synchronize(self.rp.device)

    def run(self, rounds: int) -> None:
        for _ in range(rounds):
            self.round()

    def check_errors(self) -> None:
        e = int(self.err.item())
        if e:
            raise RuntimeError(f"concurrent driver: pending list overflow (err={e})")
        self.eng.check_errors()
