"""MI355X-native batched actor group.

The reference runs one process per actor, each doing batch-1 inference of two nets on its own
GPU context with 4 blocking D2H copies per env step (actor.py:96-106, model.py:68-69; SURVEY
§3.2, P2).  Here ONE actor group drives E environments on a GPU:

* envs are vectorised on the device (``VecSyntheticAtari`` / ``VecCartPole``) or fed from CPU;
* inference for all E envs and BOTH nets is a handful of launches: the fused uint8 torso kernel,
  one x-projection GEMM per net, one LSTM step launch covering both nets (two chains), the head
  GEMM + fused dueling epilogue;
* epsilon-greedy with a per-env Ape-X ladder ``eps_i = 0.4^(1 + 7 i/(N-1))`` over the global env
  index (actor.py:22);
* n-step returns, double-Q initial priorities (bootstrapped from Q(s_{t+n}), fixing Q5),
  episode-end flushes with truncated returns (fixing Q3/Q4) and sequence-start marking with
  eta-mixed priorities all happen on the device; rows are written straight into the learner's
  HBM replay (each env owns one sub-ring, so episodes are contiguous);
* weights are read from the co-located learner's packed bf16 buffers (zero-copy "broadcast"
  when actor and learner share a GPU), or from a versioned ``WeightPublisher`` slot.

No host synchronisation per step: the whole env step is device-only and replays as a HIP graph
(``capture``); finished-episode returns land in a device ring drained when read.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np
import torch

from .config import R2D2Config, epsilon_ladder
from .engine.layout import ParamLayout
from .engine.replay_hbm import HBMReplay
from .ops._lib import check, kernels, ptr, stream_handle
from .ops.gemm import Gemm, gemm
from .ops.torso_lib import fused_torso_fwd_geom, torso_forward_library, torso_fwd_fused


_VP = ctypes.c_void_p


class ActArgs(ctypes.Structure):
    """Mirror of ``struct ActArgs`` (csrc/kernels/actor.hip); size checked against the .so."""
    _fields_ = [(name, _VP) for name in (
        "frames", "obs", "hs_cs", "ths_cs", "action", "reward", "done", "priority", "is_start",
        "leaves", "n_valid", "dirty", "dcount", "q_on", "q_tg")] + [
        (name, _VP * 2) for name in ("st_h", "st_c", "h_new", "c_new", "h32", "c", "h_bf")] + [
        (name, _VP) for name in (
            "h_row", "h_q", "h_a", "h_r", "h_step", "h_valid", "ep_start", "t", "head", "eps", "act",
            "env_reward", "env_done", "env_finished", "ret_ring", "ret_cnt", "ret_env", "marks",
            "pend", "pend_cnt")] + [
        ("FB", ctypes.c_longlong), ("seed", ctypes.c_ulonglong)] + [
        (name, ctypes.c_int) for name in ("E", "A", "H", "n", "T", "stride", "cap_e", "W", "wrap",
                                          "max_dirty", "R", "value_rescale", "pend_cap",
                                          "defer_D")] + [
        (name, ctypes.c_float) for name in ("gamma", "gamma_n", "prio_eps", "alpha", "vr_eps")]


class PackedWeights:
    """Own packed bf16/fp32 kernel-layout copy of a QNet (for actors not co-located with the
    learner).  ``load(state_dict)`` / ``load_flat(flat)`` repack on device."""

    def __init__(self, layout: ParamLayout, device):
        self.L = layout
        d = torch.device(device)
        self.flat = torch.zeros(layout.padded, dtype=torch.float32, device=d)
        self.bf = torch.zeros(layout.bf_numel, dtype=torch.bfloat16, device=d)
        self.f32 = torch.zeros(layout.f_numel, dtype=torch.float32, device=d)
        self.bf_index = layout.bf_index.to(d)
        self.f_index = layout.f_index.to(d)
        self.pk = layout.packed_views(self.bf, self.f32)
        self.lstm_b = torch.zeros(layout.G, dtype=torch.float32, device=d)
        self.version = -1

    def load_flat(self, flat: torch.Tensor, version: int = -1):
        self.flat.copy_(flat)
        k = kernels()
        s = stream_handle()
        check(k.r2_pack_bf16(ptr(self.flat), ptr(self.bf_index), ptr(self.bf), self.L.bf_numel, s), "pack")
        check(k.r2_gather_f32(ptr(self.flat), ptr(self.f_index), ptr(self.f32), self.L.f_numel, s), "gather")
        torch.add(self.pk["b_ih"], self.pk["b_hh"], out=self.lstm_b)
        self.version = version

    def load(self, sd, version: int = -1):
        self.L.load_state_dict(self.flat, sd)
        self.load_flat(self.flat, version)


class BatchedActor:
    def __init__(self, cfg: R2D2Config, replay: HBMReplay, env, online, target,
                 global_env_offset: int = 0, total_envs: Optional[int] = None, seed: int = 0):
        """online/target: objects with ``pk`` (packed views) and ``lstm_b`` -- a LearnerEngine
        (use ``engine_weights(engine)``) or ``PackedWeights``."""
        self.cfg, self.replay, self.env = cfg, replay, env
        self.online, self.target = online, target
        rc, m = cfg.replay, cfg.model
        self.E = E = env.E
        if E != replay.n_sub:
            raise ValueError(f"one sub-ring per env: env.E={E} replay.n_sub={replay.n_sub}")
        if E > 256:
            raise ValueError("an actor group drives <= 256 envs (one LSTM launch)")
        self.device = d = replay.device
        self.H, self.A, self.n = m.hidden, m.n_actions, rc.n_step
        self.T, self.stride = rc.seq_len, rc.overlap
        self.gamma = cfg.learner.gamma
        self.gamma_n = self.gamma ** self.n
        self.layout = ParamLayout(m, cfg.env)
        # fused torso forward: Atari 4x84x84 and DMLab-30 3x72x96 (else the library convs)
        self.fwd_geom = fused_torso_fwd_geom(cfg.env, m) if self.device.type == "cuda" else None
        self.fused_torso = self.fwd_geom is not None
        total = total_envs or E
        eps = [epsilon_ladder(global_env_offset + i, total, cfg.actor.eps_base, cfg.actor.eps_alpha)
               for i in range(E)]
        self.eps = torch.tensor(eps, dtype=torch.float32, device=d)
        # epsilon-greedy draws: counter-based hash of (seed, step, env) inside actor_pre_kernel
        self.seed = ((seed + 7919 * global_env_offset) * 0x9E3779B97F4A7C15 + 1) & ((1 << 64) - 1)
        H, A, n = self.H, self.A, self.n
        z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device=d)  # noqa: E731
        # recurrent state of both nets: bf16 h (MFMA operand), fp32 h (stored state), fp32 c
        self.h_bf = {k: z(E, H, dt=torch.bfloat16) for k in ("on", "tg")}
        self.h32 = {k: z(E, H) for k in ("on", "tg")}
        self.c = {k: z(E, H) for k in ("on", "tg")}
        self.h_bf_new = {k: z(E, H, dt=torch.bfloat16) for k in ("on", "tg")}
        self.h32_new = {k: z(E, H) for k in ("on", "tg")}
        self.c_new = {k: z(E, H) for k in ("on", "tg")}
        self.q = {k: z(E, A) for k in ("on", "tg")}
        self.Xn = {k: z(E, self.layout.D, dt=torch.bfloat16) for k in ("on", "tg")}
        self.xp = {k: z(E, self.layout.G) for k in ("on", "tg")}
        self.zh = {k: z(E, 2 * self.layout.HD, dt=torch.bfloat16) for k in ("on", "tg")}
        self.ctr = z(int(kernels().r2_lstm_persist_ctr_words()), dt=torch.int32)
        self.err = z(1, dt=torch.int32)
        # n-step history ring (device)
        # each env's history rows point into its own sub-ring (initially its first row), so the
        # masked scatters below never see two envs on one row
        self.h_row = (torch.arange(E, device=d, dtype=torch.int64) * replay.cap_e).repeat(n, 1)
        self.h_q = z(n, E, A)
        self.h_a = z(n, E, dt=torch.int64)
        self.h_r = z(n, E)
        self.h_step = torch.full((n, E), -1, dtype=torch.int64, device=d)
        self.h_valid = z(n, E, dt=torch.bool)
        # episode bookkeeping.  The step counter and the common sub-ring write position live on
        # the device (t_d, head_d) so one captured graph serves every step; host mirrors (t, head)
        # only pick the graph variant (the sub-ring wrap step also invalidates the old windows).
        self.t = 0                                  # actor step counter (all envs in lockstep)
        self.head = 0                               # common sub-ring write position
        self.t_d = z(1, dt=torch.int64)
        self.head_d = z(1, dt=torch.int64)
        self.ep_start = z(E, dt=torch.int64)        # actor step at which each episode started
        self.base = torch.arange(E, device=d, dtype=torch.int64) * replay.cap_e
        W = self.T + n
        self.tail_off = torch.arange(replay.cap_e - W + 1, replay.cap_e, device=d)
        # finished-episode returns: device ring + count, drained into a host list on read
        self.R = max(int(cfg.actor.return_ring), E)
        if ctypes.sizeof(ActArgs) != kernels().r2_actor_args_bytes():
            raise RuntimeError("ActArgs layout differs from csrc/kernels/actor.hip")
        self.act = z(E, dt=torch.int64)
        self.marks = z(E * (n + 2), dt=torch.int32)
        self.ret_ring = z(self.R + 1)
        self.ret_cnt = z(1, dt=torch.int64)
        self.ret_env = z(self.R + 1, dt=torch.int32)
        self._ret_read = 0
        self._returns = []
        self._return_envs = []
        self.global_env_offset = int(global_env_offset)
        self.eps_host = [float(x) for x in eps]
        self.env_steps = 0
        self.graphs = None
        # concurrent topology (engine/concurrent.py): start edits go to one of two pending lists
        # (round parity) instead of the tree, and the LSTM runs as the plain step kernel (no
        # persistent co-residency requirement on the actor's few CUs)
        self.defer = None            # dict(pend=[2 x int32], cnt=[2 x int32], cap, D)
        self.lstm_step = False
        self.n_workers = 256         # torso workgroups (grid-stride over frames)
        if hasattr(env, "reset_all"):
            env.reset_all()

    def set_weights(self, online, target) -> None:
        """Point inference at other packed weights (captured graphs must be re-captured)."""
        self.online, self.target = online, target
        self.graphs = None

    def enable_deferred(self, pend, cnt, cap: int, lookahead: int) -> None:
        """Deferred (concurrent) mode: ``pend``/``cnt`` = two pending lists + counts (round
        parity); rows are invalidated ``lookahead`` steps ahead of the write head."""
        if self.replay.cap_e <= lookahead + self.T + self.n:
            raise ValueError(f"sub-ring of {self.replay.cap_e} rows too small for lookahead {lookahead}")
        self.defer = dict(pend=pend, cnt=cnt, cap=int(cap), D=int(lookahead))
        self.lstm_step = True
        self.graphs = None

    @property
    def finished_returns(self):
        """Returns of the episodes finished so far (host list; syncs to drain the device ring,
        keeping at most ``actor.return_ring`` returns per drain)."""
        cnt = int(self.ret_cnt.item())
        lo = max(self._ret_read, cnt - self.R)
        if cnt > lo:
            ring = self.ret_ring[: self.R].cpu()
            envs = self.ret_env[: self.R].cpu()
            self._returns.extend(float(ring[i % self.R]) for i in range(lo, cnt))
            self._return_envs.extend(int(envs[i % self.R]) for i in range(lo, cnt))
        self._ret_read = cnt
        return self._returns

    def returns_by_epsilon(self, last: int = 256, buckets: int = 4) -> Dict[str, float]:
        """Mean return of the last ``last`` finished episodes per epsilon bucket (the Ape-X ladder
        split into ``buckets`` contiguous env ranges, keyed by the bucket's mean epsilon): the
        reference prints every actor's return next to its fixed epsilon (actor.py:109-110)."""
        rets = self.finished_returns[-last:]
        envs = self._return_envs[-len(rets):] if rets else []
        out: Dict[str, list] = {}
        for r, e in zip(rets, envs):
            b = min(buckets - 1, e * buckets // max(self.E, 1))
            lo_, hi_ = b * self.E // buckets, max(b * self.E // buckets + 1, (b + 1) * self.E // buckets)
            key = f"{sum(self.eps_host[lo_:hi_]) / (hi_ - lo_):.3g}"
            out.setdefault(key, []).append(r)
        return {k: float(np.mean(v)) for k, v in sorted(out.items(), key=lambda kv: -float(kv[0]))}

    # ------------------------------------------------------------------ inference
    def _infer(self):
        """Q values + next recurrent state of both nets for the current observations: one launch
        per stage for BOTH nets (torso multi-job, x-projection GEMM, 2-chain LSTM step, head
        GEMM, dueling epilogue) -- the actor step is launch-bound at these batch sizes."""
        k = kernels()
        s = stream_handle()
        E, H, L = self.E, self.H, self.layout
        nets = (("on", self.online), ("tg", self.target))
        if self.fused_torso:
            self._tjobs = np.asarray(
                [[0, E, ptr(w.pk["conv1"]), ptr(w.pk["b1"]), ptr(w.pk["conv2"]), ptr(w.pk["b2"]),
                  ptr(w.pk["conv3"]), ptr(w.pk["b3"]), ptr(self.Xn[key]), 0, 0, 0] for key, w in nets],
                dtype=np.int64)
            torso_fwd_fused(self.env.frames.reshape(E, -1), self._tjobs, self.fwd_geom,
                            self.n_workers, s)
        else:
            for key, w in nets:
                torso_forward_library(self.env.frames.reshape(E, -1), None, L, w.flat, self.cfg.env,
                                      self.cfg.model, self.Xn[key])
        gemm(*[Gemm(self.Xn[key], w.pk["w_ih"].t(), self.xp[key], bias=w.lstm_b) for key, w in nets])
        if self.lstm_step:
            # plain step kernel (lstm.hip, <= 128 rows per chain): no inter-workgroup hand-off,
            # so it runs on any CU subset; E > 128 is split into two row halves per net
            Bc = E if E <= 128 else (E + 1) // 2
            if E > 128 and (E % 2 or Bc > 128):
                raise ValueError("step-kernel LSTM: E <= 128 or an even E <= 256")
            G = self.layout.G
            rows = [(r0, Bc) for r0 in range(0, E, Bc)]
            self._chains = np.asarray(
                [[ptr(self.xp[key]) + r0 * G * 4, ptr(w.pk["w_hh"]), ptr(self.h_bf[key]) + r0 * H * 2,
                  ptr(self.c[key]) + r0 * H * 4, ptr(self.h_bf_new[key]) + r0 * H * 2,
                  ptr(self.c_new[key]) + r0 * H * 4, ptr(self.h32_new[key]) + r0 * H * 4, 0, 0]
                 for key, w in nets for r0, _ in rows], dtype=np.int64)
            check(k.r2_lstm_fwd(self._chains.ctypes.data, len(self._chains), Bc, 1, H, 0, s),
                  "lstm_step_kernel")
        else:
            self._chains = np.asarray(
                [[ptr(self.xp[key]), ptr(w.pk["w_hh"]), ptr(self.h_bf[key]), ptr(self.c[key]),
                  ptr(self.h_bf_new[key]), ptr(self.c_new[key]), ptr(self.h32_new[key]), 0, 0]
                 for key, w in nets], dtype=np.int64)
            check(k.r2_lstm_fwd_persist(self._chains.ctypes.data, 2, E, 1, H, ptr(self.ctr),
                                        ptr(self.err), s), "lstm_step")
        gemm(*[Gemm(self.h_bf_new[key], w.pk["head1"].t(), self.zh[key]) for key, w in nets])
        self._djobs = np.asarray(
            [[ptr(self.zh[key]), ptr(w.pk["head_b1"]), ptr(w.pk["head_w2"]), ptr(w.pk["head_b2"]),
              ptr(self.q[key]), 0, E] for key, w in nets], dtype=np.int64)
        check(k.r2_dueling_fwd_multi(self._djobs.ctypes.data, 2, self.A, L.HD, s), "dueling_fwd")

    # ------------------------------------------------------------------ one env step
    @property
    def can_capture(self) -> bool:
        return (self.device.type == "cuda" and self.fused_torso
                and getattr(self.env, "capture_safe", False))

    def capture(self, warmup: int = 1):
        """Capture the env step into two HIP graphs (plain step / sub-ring wrap step).  The
        warmup steps are real steps; capture itself executes nothing."""
        for _ in range(warmup):
            self.step()
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        gens = [self.env.g] if hasattr(self.env, "g") else []
        graphs, pool = {}, None
        # variants: (sub-ring wrap step?, pending-list parity) -- parity only in deferred mode
        for parity in ((0, 1) if self.defer else (0,)):
            for wrap in (False, True):
                g = torch.cuda.CUDAGraph()
                for gen in gens:
                    g.register_generator_state(gen)
                with torch.cuda.graph(g, pool=pool, stream=side):
                    self._body(wrap, parity)
                pool = g.pool()
                graphs[(wrap, parity)] = g
        torch.cuda.current_stream(self.device).wait_stream(side)
        self.graphs = graphs

    @torch.no_grad()
    def step(self, parity: int = 0):
        """One env step of every env.  ``parity``: pending list of the current round (deferred)."""
        wrap = self.head == 0
        if self.graphs is not None:
            self.graphs[(wrap, parity if self.defer else 0)].replay()
        else:
            self._body(wrap, parity)
        rp = self.replay
        self.t += 1
        self.head = (self.head + 1) % rp.cap_e
        rp.total_written += self.E
        self.env_steps += self.E

    def _args(self, wrap: bool, parity: int = 0) -> ActArgs:
        rp, rc, lc = self.replay, self.cfg.replay, self.cfg.learner
        pre = rc.stored_state == "pre"
        a = ActArgs()
        for name, t in (("frames", rp.frames), ("obs", self.env.frames), ("hs_cs", rp.hs_cs),
                        ("ths_cs", rp.target_hs_cs), ("action", rp.action), ("reward", rp.reward),
                        ("done", rp.done), ("priority", rp.priority), ("is_start", rp.is_start),
                        ("leaves", rp.tree), ("n_valid", rp.n_valid), ("dirty", rp.dirty),
                        ("dcount", rp.dirty_count), ("q_on", self.q["on"]), ("q_tg", self.q["tg"]),
                        ("h_row", self.h_row), ("h_q", self.h_q), ("h_a", self.h_a), ("h_r", self.h_r),
                        ("h_step", self.h_step), ("h_valid", self.h_valid), ("ep_start", self.ep_start),
                        ("t", self.t_d), ("head", self.head_d), ("eps", self.eps), ("act", self.act),
                        ("ret_ring", self.ret_ring), ("ret_cnt", self.ret_cnt), ("ret_env", self.ret_env),
                        ("marks", self.marks)):
            setattr(a, name, ptr(t))
        for i, key in enumerate(("on", "tg")):
            a.st_h[i] = ptr(self.h32[key] if pre else self.h32_new[key])
            a.st_c[i] = ptr(self.c[key] if pre else self.c_new[key])
            a.h_new[i], a.c_new[i] = ptr(self.h32_new[key]), ptr(self.c_new[key])
            a.h32[i], a.c[i], a.h_bf[i] = ptr(self.h32[key]), ptr(self.c[key]), ptr(self.h_bf[key])
        a.FB, a.seed = rp.frames.shape[1] if rp.frame_bytes else 0, self.seed
        a.E, a.A, a.H, a.n, a.T, a.stride = self.E, self.A, self.H, self.n, self.T, self.stride
        a.cap_e, a.W, a.wrap = rp.cap_e, self.T + self.n, int(wrap)
        a.max_dirty, a.R, a.value_rescale = rp.max_dirty, self.R, int(lc.value_rescale)
        if self.defer:
            a.pend, a.pend_cnt = ptr(self.defer["pend"][parity]), ptr(self.defer["cnt"][parity])
            a.pend_cap, a.defer_D = self.defer["cap"], self.defer["D"]
        a.gamma, a.gamma_n = self.gamma, self.gamma_n
        a.prio_eps, a.alpha, a.vr_eps = rc.priority_eps, rc.alpha, lc.value_rescale_eps
        return a

    def _body(self, wrap: bool, parity: int = 0):
        """One env step for all E envs, device-only (no host sync, capture-safe): inference of
        both nets, then actor.hip's fused bookkeeping around the device env step."""
        k = kernels()
        s = stream_handle()
        if self.cfg.actor.reset_state_every_step:   # ablation: memoryless acting
            for key in ("on", "tg"):
                self.h_bf[key].zero_()
                self.h32[key].zero_()
                self.c[key].zero_()
        self._infer()
        a = self._args(wrap, parity)
        check(k.r2_actor_pre(ctypes.byref(a), s), "actor_pre")
        reward, done, finished = self.env.step(self.act)
        a.env_reward, a.env_finished = ptr(reward.float().contiguous()), ptr(finished.contiguous())
        a.env_done = ptr(done.to(torch.bool).contiguous())
        check(k.r2_actor_post(ctypes.byref(a), s), "actor_post")
        if not self.defer:   # deferred: the learner's stream applies the pending list
            self.replay.mark_starts(self.marks)
            self.replay.update_tree()
        check(k.r2_actor_tail(ctypes.byref(a), s), "actor_tail")

    def run(self, n_steps: int):
        for _ in range(n_steps):
            self.step()


def engine_weights(engine):
    """Adapter exposing a LearnerEngine's live online / target packed weights to an actor."""

    class _W:
        def __init__(self, pk, b, flat):
            self.pk, self.lstm_b, self.flat = pk, b, flat

    return (_W(engine.pk, engine.lstm_b, engine.master),
            _W(engine.pk_t, engine.lstm_b_t, engine.target))
