"""Reference-compatible actor role.

Parity target: ``/root/reference/actor.py`` -- ``actor_process(actor_id, n_actors, shared_dict,
device)`` and ``class Actor`` with ``run / step / select_action / reset / load_model /
calc_priority / set_seq_start_index``; Ape-X epsilon ladder; n-step transitions carrying the
stored recurrent state of the online and target nets; episode segmentation into overlapping
sequences with eta-mixed priorities; replay shipped to the learner every
``memory_save_interval`` episodes; weights pulled every ``net_load_interval`` episodes.

This single-env actor is the compatibility path (one process per actor, like the reference).
The MI355X-native actor is ``actor_batched.BatchedActor``: hundreds of envs per GPU with batched
HIP inference writing straight into the HBM replay.

Fixes (each switchable back through ``cfg`` / ``legacy=True`` for comparison):
  Q1  epsilon ladder for a single actor is 0.4 (reference divides by zero)
  Q3/Q4 n-step transitions: first transition kept, tail returns correctly truncated
  Q5  the n-step priority bootstraps from Q(s_{t+n}), not Q(s_{t+n-1})
  Q6  ``replay.stored_state = "pre"`` stores the state *before* consuming o_t (paper); "post"
      (default of the reference preset) keeps the reference behaviour
  Q12 sequence start indices are wrapped into the ring
  Q13 no blocking D2H per forward beyond the action / q-values the actor needs anyway
"""
from __future__ import annotations

import gc
import os
from typing import Optional

import numpy as np
import torch

from .config import R2D2Config, epsilon_ladder, get_config
from .envs import make_env
from .models.qnet import QNet
from .replay.memory import ReplayMemory
from .replay.nstep import NStepMemory


def actor_process(actor_id, n_actors, shared_dict, device="cuda:0", cfg: Optional[R2D2Config] = None,
                  max_steps: Optional[int] = None, max_episodes: Optional[int] = None,
                  memory_path: Optional[str] = None, beat=None, shm_ring: Optional[str] = None,
                  shm_weights: Optional[str] = None, seed: int = 0):
    """Actor process entry.  ``beat``: supervisor heartbeat (utils/supervisor.py).  Native
    transport (main.py --mode native --cpu-actors N): ``shm_ring`` = name of this actor's
    shared-memory trajectory ring into the learner's HBM replay, ``shm_weights`` = the learner's
    shared-memory weight slot (seqlock); without them the reference file / Manager-dict transport."""
    if isinstance(device, str) and device.startswith("cuda") and not torch.cuda.is_available():
        device = "cpu"
    if str(device) == "cpu":
        # one intra-op thread per CPU actor process by default: N actors x the machine's cores
        # threads each would oversubscribe the host many times over
        torch.set_num_threads(int(os.environ.get("R2D2_ACTOR_THREADS", "1")))
    actor = Actor(actor_id, n_actors, shared_dict, device, cfg=cfg, memory_path=memory_path, seed=seed)
    if shm_ring:
        from .parallel.trajectory import ShmTrajectoryWriter
        actor.transport = ShmTrajectoryWriter(shm_ring)
    if shm_weights:
        from .parallel.weights import ShmWeightsReader
        actor.weights_reader = ShmWeightsReader(shm_weights, actor.cfg)
    actor.run(max_steps=max_steps, max_episodes=max_episodes, beat=beat)


class Actor:
    def __init__(self, actor_id, n_actors, shared_dict, device="cpu", cfg: Optional[R2D2Config] = None,
                 env=None, memory_path: Optional[str] = None, legacy: bool = False, seed: int = 0):
        cfg = cfg or get_config("reference")
        self.cfg = cfg
        rc, ac, lc = cfg.replay, cfg.actor, cfg.learner
        self.legacy = legacy
        # params (actor.py:20-27)
        self.gamma = lc.gamma
        self.epsilon = epsilon_ladder(actor_id, n_actors, ac.eps_base, ac.eps_alpha)
        self.bootstrap_steps = rc.n_step
        self.alpha = rc.alpha
        self.priority_epsilon = rc.priority_eps
        self.device = device
        self.actor_id = actor_id
        self.memory_path = memory_path or os.path.join(".", "logs", "memory")
        # memory (actor.py:33-47)
        self.memory_size = ac.local_capacity
        self.batch_size = 32
        self.action_repeat = cfg.env.action_repeat
        self.n_stacks = cfg.env.n_stacks
        self.burn_in_length = rc.burn_in
        self.learning_length = rc.learn
        self.overlap_length = rc.overlap
        self.eta = rc.eta
        self.sequence_length = self.burn_in_length + self.learning_length
        self.stack_count = max(1, self.n_stacks // self.action_repeat)
        self.memory_save_interval = ac.memory_save_interval
        self.episode_start_index = 0
        self.n_steps_memory = NStepMemory(self.bootstrap_steps, self.gamma, legacy=legacy)
        self.replay_memory = self._new_memory()
        # net (actor.py:49-54)
        self.shared_dict = shared_dict
        self.net_load_interval = ac.net_load_interval
        self.net = QNet(device, cfg.model, cfg.env).to(device)
        self.target_net = QNet(device, cfg.model, cfg.env).to(device)
        self.target_net.load_state_dict(self.net.state_dict())
        self.weights_version = -1
        # env (actor.py:56-62)
        self.env = env if env is not None else make_env(cfg, seed=seed + actor_id)
        self.rng = np.random.default_rng(seed + 1000 + actor_id)
        self.episode_reward = 0.0
        self.n_episodes = 0
        self.n_steps = 0
        self.total_steps = 0
        self.memory_count = 0
        self.episode_returns = []
        self.transport = None           # ShmTrajectoryWriter (native) | None (reference files)
        self.weights_reader = None      # ShmWeightsReader (native) | None (Manager dict)
        self.pushed_rows = 0
        self.state = self.env.reset()

    def _new_memory(self) -> ReplayMemory:
        e, m, rc = self.cfg.env, self.cfg.model, self.cfg.replay
        if m.torso == "atari":
            return ReplayMemory(self.memory_size, self.batch_size, self.bootstrap_steps,
                                (e.frame_h, e.frame_w), m.hidden, self.action_repeat, self.n_stacks,
                                burn_in=rc.burn_in, learning=rc.learn, eta=rc.eta, legacy=self.legacy,
                                obs_shape=(e.channels_per_frame * e.n_stacks, e.frame_h, e.frame_w))
        return ReplayMemory(self.memory_size, self.batch_size, self.bootstrap_steps, cell_size=m.hidden,
                            action_repeat=1, n_stacks=1, burn_in=rc.burn_in, learning=rc.learn,
                            eta=rc.eta, legacy=self.legacy, obs_shape=(e.obs_dim * e.n_stacks,),
                            obs_dtype=np.float32)

    # ------------------------------------------------------------------ loop
    def run(self, max_steps: Optional[int] = None, max_episodes: Optional[int] = None, beat=None):
        from .utils.faults import Liveness
        live = Liveness("actor", self.actor_id, beat)
        while True:
            if max_steps is not None and self.total_steps >= max_steps:
                break
            if max_episodes is not None and self.n_episodes >= max_episodes:
                break
            live.tick(self.total_steps)
            self.step()
        self.flush()

    def _emit(self, q_boot, tq_boot, done):
        pre_q, state, h, c, th, tc, action, reward, stack_count = self.n_steps_memory.get()
        priority = self.calc_priority(pre_q, action, reward, q_boot, tq_boot, done)
        self.replay_memory.add(state, h, c, th, tc, action, reward, done, stack_count, priority)
        self.memory_count += 1

    def step(self):
        state = self.state
        action, q_value, h, c, target_q_value, target_h, target_c = self.select_action(state)
        q_value = q_value.detach().cpu().numpy()
        target_q_value = target_q_value.detach().cpu().numpy()
        if not self.legacy and self.n_steps_memory.size >= self.bootstrap_steps:
            # window of the oldest transition is complete; bootstrap from Q(s_t) (fix Q5)
            self._emit(q_value, target_q_value, False)
        next_state, reward, done, _ = self.env.step(action)
        self.episode_reward += reward
        self.n_steps += 1
        self.total_steps += 1
        frames = state[-self.action_repeat:] if self.cfg.model.torso == "atari" else state
        self.n_steps_memory.add(q_value, frames, h, c, target_h, target_c, action, reward,
                                self.stack_count)
        if self.stack_count > 1:
            self.stack_count -= 1
        if self.legacy and self.n_steps > self.bootstrap_steps:   # actor.py:81-85 (Q3/Q5)
            self._emit(q_value, target_q_value, done)
        self.state = np.array(next_state, copy=True)
        if done:
            while self.n_steps_memory.size > 0:                   # actor.py:88-93
                self._emit(q_value, target_q_value, True)
            self.reset()

    def select_action(self, state):
        """actor.py:96-106: both nets step on the same observation; epsilon-greedy on online Q."""
        x = torch.as_tensor(np.asarray(state), dtype=torch.float32).unsqueeze(0).to(self.device)
        pre = self.cfg.replay.stored_state == "pre"
        if pre:
            h_pre, c_pre = self._state_of(self.net)
            th_pre, tc_pre = self._state_of(self.target_net)
        with torch.no_grad():
            q_value, h, c = self.net(x, True)
            target_q_value, target_h, target_c = self.target_net(x, True)
        if pre:
            h, c, target_h, target_c = h_pre, c_pre, th_pre, tc_pre
        if self.rng.random() < self.epsilon:
            action = int(self.rng.integers(self.cfg.model.n_actions))
        else:
            action = int(q_value.argmax().item())
        return action, q_value, h, c, target_q_value, target_h, target_c

    def _state_of(self, net):
        H = self.cfg.model.hidden
        if net.hs is None:
            z = np.zeros((1, H), dtype=np.float32)
            return z, z.copy()
        return (torch.as_tensor(net.hs).detach().cpu().numpy().reshape(1, H),
                torch.as_tensor(net.cs).detach().cpu().numpy().reshape(1, H))

    def reset(self):
        """actor.py:108-135."""
        self.episode_returns.append(self.episode_reward)
        print("episodes:", self.n_episodes, "actor_id:", self.actor_id, "return:", self.episode_reward,
              flush=True)
        self.net.reset()
        self.target_net.reset()
        self.set_seq_start_index()
        self.state = self.env.reset()
        self.episode_start_index = self.replay_memory.index
        self.episode_reward = 0.0
        self.n_episodes += 1
        self.n_steps = 0
        self.memory_count = 0
        self.stack_count = max(1, self.n_stacks // self.action_repeat)
        self.n_steps_memory = NStepMemory(self.bootstrap_steps, self.gamma, legacy=self.legacy)
        if self.n_episodes % self.memory_save_interval == 0:
            self.flush()
        if self.n_episodes % self.net_load_interval == 0:
            self.load_model()

    def flush(self) -> None:
        """Ship the local replay to the learner (replay_memory.py:125-152 file save, or one record
        into the shared-memory ring of the native transport) and start a new one."""
        if self.replay_memory.size == 0:
            return
        if self.transport is not None:
            from .utils.faults import faults
            mem = {k: v[: self.replay_memory.size] for k, v in self.replay_memory.memory.items()}
            if not faults().drop("push", self.actor_id):
                self.transport.push(mem)
                self.pushed_rows += self.replay_memory.size
        else:
            self.replay_memory.save(self.memory_path, self.actor_id)
        self.replay_memory = self._new_memory()
        self.episode_start_index = 0
        gc.collect()

    def load_model(self):
        """actor.py:137-142; reads a consistent (net, target) pair published under one version."""
        if self.weights_reader is not None:
            got = self.weights_reader.fetch(self.weights_version)
            if got is not None:
                sd_on, sd_tg, v = got
                self.net.load_state_dict(sd_on)
                self.target_net.load_state_dict(sd_tg)
                self.weights_version = v
            return got is not None
        try:
            sd = self.shared_dict
            self.net.load_state_dict(sd["net_state"])
            self.target_net.load_state_dict(sd["target_net_state"])
            self.weights_version = int(sd.get("version", -1)) if hasattr(sd, "get") else -1
            return True
        except (KeyError, RuntimeError, TypeError) as e:
            print(f"load error: {e!r}", flush=True)
            return False

    def calc_priority(self, q_value, action, reward, next_q_value, target_next_q_value, done):
        """actor.py:144-157 (double-Q n-step TD error -> (|delta|+eps)^alpha)."""
        q_value = np.asarray(q_value).reshape(-1)[action]
        target_next_q_value = np.asarray(target_next_q_value).reshape(-1)
        if done:
            target_q_value = reward
        else:
            next_action = int(np.asarray(next_q_value).reshape(-1).argmax())
            target_q_value = reward + (self.gamma ** self.bootstrap_steps) * target_next_q_value[next_action]
        priority = np.abs(q_value - target_q_value) + self.priority_epsilon
        return float(priority ** self.alpha)

    def set_seq_start_index(self):
        """actor.py:159-167: starts every `overlap` rows plus a final start T rows before the end
        (Q12: wrapped into the ring; episodes shorter than T contribute no sequence)."""
        last_index = self.replay_memory.index
        start_index = self.episode_start_index
        T = self.sequence_length
        if last_index - start_index < T and not self.legacy:
            return
        seq = list(range(start_index, last_index - T, self.overlap_length))
        seq.append(last_index - T)
        seq = np.array(seq, dtype=np.int64)
        if not self.legacy:
            seq = np.unique(seq % self.replay_memory.memory_size)
        self.replay_memory.memory["is_seq_start"][seq] = 1
        self.replay_memory.update_sequence_priority(seq)
