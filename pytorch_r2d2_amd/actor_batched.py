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

No host synchronisation per step except the optional episode-return logging.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from .config import R2D2Config, epsilon_ladder
from .engine.layout import ParamLayout
from .engine.learner_engine import addmm_f32
from .engine.replay_hbm import HBMReplay
from .ops._lib import check, kernels, ptr, stream_handle
from .ops.torso_lib import fused_torso_supported, torso_forward_library


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
        self.fused_torso = fused_torso_supported(cfg.env, m)
        total = total_envs or E
        eps = [epsilon_ladder(global_env_offset + i, total, cfg.actor.eps_base, cfg.actor.eps_alpha)
               for i in range(E)]
        self.eps = torch.tensor(eps, dtype=torch.float32, device=d)
        self.g = torch.Generator(device=d)
        self.g.manual_seed(seed + 7919 * global_env_offset)
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
        self.X = z(E, self.layout.D, dt=torch.bfloat16)
        self.ctr = z(int(kernels().r2_lstm_persist_ctr_words()), dt=torch.int32)
        self.err = z(1, dt=torch.int32)
        # n-step history ring (device)
        self.h_row = z(n, E, dt=torch.int64)
        self.h_q = z(n, E, A)
        self.h_a = z(n, E, dt=torch.int64)
        self.h_r = z(n, E)
        self.h_step = torch.full((n, E), -1, dtype=torch.int64, device=d)
        self.h_valid = z(n, E, dt=torch.bool)
        # episode bookkeeping
        self.t = 0                                  # actor step counter (all envs in lockstep)
        self.head = 0                               # common sub-ring write position
        self.ep_start = z(E, dt=torch.int64)        # actor step at which each episode started
        self.base = torch.arange(E, device=d, dtype=torch.int64) * replay.cap_e
        self.finished_returns = []
        self.env_steps = 0
        if hasattr(env, "reset_all"):
            env.reset_all()

    # ------------------------------------------------------------------ inference
    def _infer(self):
        """Q values + next recurrent state of both nets for the current observations."""
        k = kernels()
        s = stream_handle()
        E, H, L = self.E, self.H, self.layout
        for key, w in (("on", self.online), ("tg", self.target)):
            pk = w.pk
            if self.fused_torso:
                check(k.r2_torso_fwd(ptr(self.env.frames), 0, E, ptr(pk["conv1"]), ptr(pk["b1"]),
                                     ptr(pk["conv2"]), ptr(pk["b2"]), ptr(pk["conv3"]), ptr(pk["b3"]),
                                     ptr(self.X), 0, 0, 256, s), "torso_fwd")
            else:
                torso_forward_library(self.env.frames.reshape(E, -1), None, L, w.flat, self.cfg.env,
                                      self.cfg.model, self.X)
            xp = addmm_f32(w.lstm_b, self.X, pk["w_ih"].t())
            chain = [ptr(xp), ptr(pk["w_hh"]), ptr(self.h_bf[key]), ptr(self.c[key]),
                     ptr(self.h_bf_new[key]), ptr(self.c_new[key]), ptr(self.h32_new[key]), 0, 0]
            arr = np.asarray(chain, dtype=np.int64)
            check(k.r2_lstm_fwd_persist(arr.ctypes.data, 1, E, 1, H, ptr(self.ctr), ptr(self.err), s),
                  "lstm_step")
            zz = torch.mm(self.h_bf_new[key], pk["head1"].t())
            check(k.r2_dueling_fwd(ptr(zz), ptr(pk["head_b1"]), ptr(pk["head_w2"]), ptr(pk["head_b2"]),
                                   ptr(self.q[key]), 0, E, self.A, L.HD, s), "dueling_fwd")

    # ------------------------------------------------------------------ one env step
    @torch.no_grad()
    def step(self):
        E, n, d = self.E, self.n, self.device
        rp, rc = self.replay, self.cfg.replay
        rows = self.base + self.head                                    # (E,) this step's rows
        # the rows we are about to write stop being sequence starts; at a sub-ring wrap also the
        # old sequences whose window wraps into the rows we start overwriting
        clear = rows
        if self.head == 0 and rp.total_written > 0:
            W = self.T + n
            tail = torch.arange(rp.cap_e - W + 1, rp.cap_e, device=d)
            clear = torch.cat([rows, (self.base[:, None] + tail[None, :]).reshape(-1)])
        rp.clear_rows(clear)
        # observation frames of this step -> replay rows (state uint8, like state*255)
        rp.frames[rows] = self.env.frames
        pre = rc.stored_state == "pre"
        self._infer()
        q_on, q_tg = self.q["on"], self.q["tg"]
        for key, buf in (("on", rp.hs_cs), ("tg", rp.target_hs_cs)):
            h = self.h32[key] if pre else self.h32_new[key]
            c = self.c[key] if pre else self.c_new[key]
            buf[rows] = torch.cat([h, c], 1)
        # ---- finalise the transition of step t-n (its n rewards are known; bootstrap Q(s_t))
        slot = self.t % n
        a_star = q_on.argmax(1, keepdim=True)
        boot = q_tg.gather(1, a_star).squeeze(1)
        self._finalize_slot(slot, boot)
        # ---- act (epsilon-greedy) and step the envs
        rand = torch.rand(E, device=d, generator=self.g)
        ra = torch.randint(0, self.A, (E,), device=d, generator=self.g)
        action = torch.where(rand < self.eps, ra, q_on.argmax(1))
        rp.action[rows] = action.to(torch.uint8)
        reward, done, finished = self.env.step(action)
        self.h_row[slot], self.h_q[slot], self.h_a[slot] = rows, q_on, action
        self.h_r[slot] = reward
        self.h_step[slot] = self.t
        self.h_valid[slot] = True
        # ---- mark the start whose window just became complete (rows finalised through t-n)
        newest = (self.t - n) - self.ep_start                           # newest finalised offset
        o = newest - self.T + 1
        ok = (o >= 0) & (o % self.stride == 0)
        srow = self.base + (self.head - (self.t - self.ep_start) + o) % rp.cap_e
        cand = [torch.where(ok, srow, torch.full_like(srow, -1))]
        # ---- episode ends: flush pending transitions (truncated returns, done=1), final starts
        if bool(done.any()):
            cand.append(self._flush_done(done))
            fin = finished[done]
            self.finished_returns.extend(fin.tolist())
        marks = torch.cat(cand).to(torch.int32)
        rp.mark_starts(marks)
        # recurrent state advances; episodes that ended restart from zero state
        keep = (~done).float()[:, None]
        for key in ("on", "tg"):
            self.h32[key] = self.h32_new[key] * keep
            self.c[key] = self.c_new[key] * keep
            self.h_bf[key] = self.h32[key].to(torch.bfloat16)
        self.ep_start = torch.where(done, torch.full_like(self.ep_start, self.t + 1), self.ep_start)
        rp.flush_tree()
        self.t += 1
        self.head = (self.head + 1) % rp.cap_e
        rp.total_written += E
        self.env_steps += E

    def _write_final(self, rows, q_sel, ret, done_flag, valid):
        rp, rc = self.replay, self.cfg.replay
        y = ret
        delta = q_sel - y
        prio = (delta.abs() + rc.priority_eps) ** rc.alpha
        r_idx = torch.where(valid, rows, torch.zeros_like(rows))
        rp.reward[r_idx] = torch.where(valid, ret, rp.reward[r_idx])
        rp.done[r_idx] = torch.where(valid, torch.full_like(rp.done[r_idx], done_flag), rp.done[r_idx])
        rp.priority[r_idx] = torch.where(valid, prio, rp.priority[r_idx])

    def _returns_from(self, step_from: torch.Tensor, upto: int) -> torch.Tensor:
        """sum_k gamma^(s_k - step_from) r_k over buffered steps s_k in [step_from, upto]."""
        st = self.h_step                                               # (n, E)
        inside = (st >= step_from[None, :]) & (st <= upto) & (st >= 0)
        pw = torch.pow(torch.tensor(self.gamma, device=self.device),
                       (st - step_from[None, :]).clamp_min(0).float())
        return (self.h_r * pw * inside.float()).sum(0)

    def _finalize_slot(self, slot: int, boot: torch.Tensor):
        valid = self.h_valid[slot]
        s0 = self.h_step[slot]
        R = self._returns_from(s0, self.t - 1)
        if self.cfg.learner.value_rescale:
            from .models.qnet import value_rescale, value_rescale_inv
            eps = self.cfg.learner.value_rescale_eps
            y = value_rescale(R + self.gamma_n * value_rescale_inv(boot, eps), eps)
        else:
            y = R + self.gamma_n * boot
        q_sel = self.h_q[slot].gather(1, self.h_a[slot][:, None]).squeeze(1)
        rp, rc = self.replay, self.cfg.replay
        prio = ((q_sel - y).abs() + rc.priority_eps) ** rc.alpha
        rows = torch.where(valid, self.h_row[slot], torch.zeros_like(self.h_row[slot]))
        rp.reward[rows] = torch.where(valid, R, rp.reward[rows])
        rp.done[rows] = torch.where(valid, torch.zeros_like(rp.done[rows]), rp.done[rows])
        rp.priority[rows] = torch.where(valid, prio, rp.priority[rows])
        self.h_valid[slot] = False

    def _flush_done(self, done: torch.Tensor) -> torch.Tensor:
        """Episode end for envs in `done`: every pending transition gets its truncated return,
        done=1 (no bootstrap).  Returns the start rows to mark (or -1)."""
        n, t = self.n, self.t
        rp = self.replay
        for j in range(n):
            valid = self.h_valid[j] & done
            R = self._returns_from(self.h_step[j], t)
            q_sel = self.h_q[j].gather(1, self.h_a[j][:, None]).squeeze(1)
            self._write_final(self.h_row[j], q_sel, R, 1, valid)
            self.h_valid[j] = self.h_valid[j] & ~done
        # starts whose windows end inside the just-finalised tail, plus the final start L-T
        L = (t - self.ep_start) + 1                                    # episode length (rows)
        prev_newest = (t - n) - self.ep_start                          # handled by per-step marks
        out = []
        for jj in range(n + 1):
            o = L - self.T - jj
            ok = done & (o >= 0) & (o > prev_newest - self.T + 1) & ((o % self.stride == 0) | (jj == 0))
            srow = self.base + (self.head - (t - self.ep_start) + o) % rp.cap_e
            out.append(torch.where(ok, srow, torch.full_like(srow, -1)))
        return torch.cat(out)

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
