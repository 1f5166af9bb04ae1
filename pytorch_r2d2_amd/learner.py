"""Reference-compatible learner role.

Parity target: ``/root/reference/learner.py`` -- ``learner_process(n_actors, shared_dict)`` and
``class Learner`` with ``run / train / interval / save_model``; cadences (target sync every 1000
steps, weight publish every 100, actor-file ingest every 20, checkpoint every 10 000), the
``save/{n}_save.pt`` checkpoint (CPU state_dict of the online net) and the ``shared_dict`` keys
``'net_state'`` / ``'target_net_state'``.

Two backends behind the same API:

* ``hip``   -- on an MI355X with the Atari torso: the HBM replay (``engine.replay_hbm``) and the
               graph-captured HIP learner step (``engine.learner_engine``).  Actor files are
               ingested straight into device memory.
* ``torch`` -- anywhere else (CPU, MLP torso / CartPole): host ``ReplayMemory`` + the fp32
               autograd learner (``learner_ref``) + torch optimizers.

Fixes: Q2 (transport files are tensor-only and never silently deleted), Q11 (``save/`` is
created), the weight publish is versioned so actors never mix net/target from different steps,
and a full-state checkpoint (optimizer, target, counters, RNG) enables ``resume``.
"""
from __future__ import annotations

import os
import time
from typing import Optional

import numpy as np
import torch

from .config import R2D2Config, get_config
from .learner_ref import SeqBatch, r2d2_loss
from .models.qnet import QNet
from .replay.memory import ReplayMemory
from .utils.checkpoint import save_full_checkpoint, save_reference_checkpoint
from .utils.metrics import MetricsLogger


def learner_process(n_actors, shared_dict, device: Optional[str] = None, cfg: Optional[R2D2Config] = None,
                    max_steps: Optional[int] = None, memory_path: Optional[str] = None,
                    metrics_path: Optional[str] = None, beat=None):
    learner = Learner(n_actors, shared_dict, device=device, cfg=cfg, memory_path=memory_path,
                      metrics_path=metrics_path)
    learner.run(max_steps=max_steps, beat=beat)


def _pick_backend(cfg: R2D2Config, device: str) -> str:
    if not str(device).startswith("cuda") or not torch.cuda.is_available():
        return "torch"
    m, e = cfg.model, cfg.env
    if m.torso == "atari" and tuple(m.conv_channels) == (32, 32, 32) and \
            (e.frame_h, e.frame_w, e.channels_per_frame * e.n_stacks) == (84, 84, 4):
        return "hip"
    return "torch"


class Learner:
    def __init__(self, n_actors, shared_dict, device: Optional[str] = None,
                 cfg: Optional[R2D2Config] = None, memory_path: Optional[str] = None,
                 metrics_path: Optional[str] = None, backend: Optional[str] = None,
                 replay_capacity: Optional[int] = None):
        cfg = cfg or get_config("reference")
        self.cfg = cfg
        rc, lc = cfg.replay, cfg.learner
        if device is None:
            device = "cuda:0" if torch.cuda.is_available() else "cpu"
        self.device = device
        self.backend = backend or _pick_backend(cfg, device)
        # params (learner.py:20-28)
        self.gamma = lc.gamma
        self.alpha = rc.alpha
        self.bootstrap_steps = rc.n_step
        self.initial_exploration = lc.initial_exploration
        self.priority_epsilon = rc.priority_eps
        self.n_epochs = 0
        self.n_actors = n_actors
        self.memory_path = memory_path or os.path.join(".", "logs", "memory")
        self.burn_in_length = rc.burn_in
        self.learning_length = rc.learn
        self.sequence_length = rc.seq_len
        self.memory_size = replay_capacity or rc.capacity
        self.batch_size = lc.batch_size
        self.memory_load_interval = lc.ingest_interval
        self.shared_dict = shared_dict
        self.net_save_interval = lc.publish_interval
        self.target_update_interval = lc.target_update_interval
        self.version = 0
        self.metrics = MetricsLogger(metrics_path) if metrics_path else None
        torch.manual_seed(cfg.seed)
        if self.backend == "hip":
            from .engine.learner_engine import LearnerEngine
            from .engine.replay_hbm import HBMReplay
            self.replay_memory = HBMReplay(cfg, device, capacity=self.memory_size,
                                           n_subrings=max(1, n_actors))
            self.engine = LearnerEngine(cfg, self.replay_memory, device)
            self.net = None
        else:
            self.replay_memory = self._new_host_memory()
            self.net = QNet(device, cfg.model, cfg.env).to(device)
            self.target_net = QNet(device, cfg.model, cfg.env).to(device)
            self.target_net.load_state_dict(self.net.state_dict())
            if lc.optimizer == "adam":
                self.optim = torch.optim.Adam(self.net.parameters(), lr=lc.lr, eps=lc.eps,
                                              betas=tuple(lc.adam_betas))
            else:  # learner.py:51
                self.optim = torch.optim.RMSprop(self.net.parameters(), lr=lc.lr, alpha=lc.rms_alpha,
                                                 eps=lc.eps, centered=True)
        self.save_model()

    def _new_host_memory(self) -> ReplayMemory:
        e, m, rc = self.cfg.env, self.cfg.model, self.cfg.replay
        if m.torso == "atari":
            return ReplayMemory(self.memory_size, self.batch_size, rc.n_step, (e.frame_h, e.frame_w),
                                m.hidden, e.action_repeat, e.n_stacks, burn_in=rc.burn_in,
                                learning=rc.learn, eta=rc.eta,
                                obs_shape=(e.channels_per_frame * e.n_stacks, e.frame_h, e.frame_w),
                                seed=self.cfg.seed)
        # the sampler's generator is seeded from the config: an unseeded one (OS entropy) made the
        # in-process CartPole run differ from run to run
        return ReplayMemory(self.memory_size, self.batch_size, rc.n_step, cell_size=m.hidden,
                            action_repeat=1, n_stacks=1, burn_in=rc.burn_in, learning=rc.learn,
                            eta=rc.eta, obs_shape=(e.obs_dim * e.n_stacks,), obs_dtype=np.float32,
                            seed=self.cfg.seed)

    # ------------------------------------------------------------------ loop (learner.py:53-66)
    def replay_size(self) -> int:
        return self.replay_memory.size

    def ingest(self) -> int:
        n = 0
        for i in range(self.n_actors):
            try:
                if self.backend == "hip":
                    n += self.replay_memory.ingest_file(self.memory_path, i)
                else:
                    n += self.replay_memory.load(self.memory_path, i)
            except Exception as e:  # keep running; the file is left in place for inspection
                print(f"ingest error actor {i}: {e!r}", flush=True)
        return n

    def run(self, max_steps: Optional[int] = None, idle_sleep: float = 0.01, beat=None):
        """learner.py:53-66, plus liveness: heartbeat + fault hooks every iteration and, on the
        HIP backend, the persistent kernels' error word at every weight publication (a timed-out
        hand-off raises instead of training on garbage state)."""
        from .utils.faults import Liveness
        live = Liveness("learner", 0, beat)
        while max_steps is None or self.n_epochs < max_steps:
            live.tick(self.n_epochs)
            if self.replay_size() > self.initial_exploration:
                self.train()
                self.n_epochs += 1
                if self.n_epochs % 100 == 0:
                    print("trained", self.n_epochs, "epochs", flush=True)
                self.interval()
            else:
                if self.ingest() == 0:
                    time.sleep(idle_sleep)

    # ------------------------------------------------------------------ train (learner.py:68-104)
    def train(self) -> float:
        if self.backend == "hip":
            self.engine.step()
            loss = None
            if self.metrics and self.n_epochs % 100 == 0:
                loss = self.engine.loss_value()
                self.metrics.log("learner", step=self.n_epochs, loss=loss)
            return loss
        cfg, rc = self.cfg, self.cfg.replay
        batch, seq_index, index, probs, n_valid = self.replay_memory.sample(self.device, return_probs=True)
        sb = self._seq_batch(batch, probs, n_valid)
        out = r2d2_loss(self.net, self.target_net, sb, cfg)
        self.optim.zero_grad()
        out["loss"].backward()
        if cfg.learner.grad_clip > 0:
            torch.nn.utils.clip_grad_norm_(self.net.parameters(), cfg.learner.grad_clip)
        self.optim.step()
        prio = out["priority"].cpu().numpy()
        self.replay_memory.update_priority(index[rc.burn_in:].reshape(-1), prio.reshape(-1))
        self.replay_memory.update_sequence_priority(seq_index, True)
        loss = float(out["loss"].item())
        if self.metrics and self.n_epochs % 100 == 0:
            self.metrics.log("learner", step=self.n_epochs, loss=loss,
                             mean_abs_td=float(out["delta"].abs().mean()))
        return loss

    def _seq_batch(self, batch, probs, n_valid) -> SeqBatch:
        rc, H = self.cfg.replay, self.cfg.model.hidden
        n, T = rc.n_step, rc.seq_len
        obs = torch.cat([batch["state"], batch["next_state"][T - n:]], 0)
        w = torch.ones(obs.shape[1], device=self.device)
        if rc.beta > 0:
            w = torch.as_tensor((n_valid * np.maximum(probs, 1e-30)) ** (-rc.beta), dtype=torch.float32,
                                device=self.device)
            w = w / w.max()
        if self.cfg.learner.target_mode == "shifted":  # target chain starts at the sequence start
            th0, tc0 = batch["target_hs0"], batch["target_cs0"]
        else:                                            # target chain on next_state (learner.py:72)
            th0, tc0 = batch["target_hs"], batch["target_cs"]
        return SeqBatch(obs=obs, h0=batch["hs"], c0=batch["cs"], th0=th0, tc0=tc0,
                        nh0=batch["next_hs"], nc0=batch["next_cs"],
                        action=batch["action"].squeeze(-1), reward=batch["reward"].squeeze(-1),
                        done=batch["done"].squeeze(-1), weights=w)

    # ------------------------------------------------------------------ interval (learner.py:106-120)
    def interval(self):
        lc = self.cfg.learner
        if self.n_epochs % self.target_update_interval == 0 and self.backend == "torch":
            self.target_net.load_state_dict(self.net.state_dict())
        if self.n_epochs % self.net_save_interval == 0:
            if self.backend == "hip":
                self.engine.check_errors()
            self.save_model()
        if self.n_epochs % self.memory_load_interval == 0:
            self.ingest()
        if self.n_epochs % lc.checkpoint_interval == 0:
            save_reference_checkpoint(self.state_dict(), self.n_epochs, lc.save_dir)

    # ------------------------------------------------------------------ weights
    def state_dict(self):
        if self.backend == "hip":
            return self.engine.state_dict()
        return {k: v.detach().cpu().clone() for k, v in self.net.state_dict().items()}

    def target_state_dict(self):
        if self.backend == "hip":
            return self.engine.target_state_dict()
        return {k: v.detach().cpu().clone() for k, v in self.target_net.state_dict().items()}

    def save_model(self):
        """learner.py:122-124 -- publish CPU state_dicts (net + target) with a version number."""
        if self.shared_dict is None:
            return
        self.version += 1
        self.shared_dict["net_state"] = self.state_dict()
        self.shared_dict["target_net_state"] = self.target_state_dict()
        self.shared_dict["version"] = self.version

    def save_checkpoint(self, path: str):
        opt = None if self.backend == "hip" else self.optim.state_dict()
        extra = {"version": torch.tensor(self.version)}
        if self.backend == "hip":
            extra.update(self.engine.full_state_extra())
        save_full_checkpoint(path, self.state_dict(), self.target_state_dict(), opt, self.n_epochs,
                             self.cfg, extra)

    def resume(self, path: str) -> int:
        """Continue from a full-state checkpoint (weights, target, optimizer state, counters, RNG;
        SURVEY §5.4).  The replay itself is not part of the checkpoint: actors refill it.
        Returns the restored learner step."""
        from .utils.checkpoint import load_full_checkpoint, restore_rng
        obj = load_full_checkpoint(path)
        restore_rng(obj)
        if self.backend == "hip":
            self.engine.load_full_state(obj)
        else:
            self.net.load_state_dict(obj["online"])
            self.target_net.load_state_dict(obj["target"])
            if obj.get("optimizer"):
                self.optim.load_state_dict(obj["optimizer"])
        self.n_epochs = int(obj["step"])
        if "version" in (obj.get("extra") or {}):
            self.version = int(obj["extra"]["version"])
        self.save_model()
        return self.n_epochs
