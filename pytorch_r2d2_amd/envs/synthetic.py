"""Synthetic Atari-shaped environments (no ROMs in this image).

Dynamics ("cue-and-act"): every ``switch`` agent steps the env draws a target action and paints
a bright vertical bar in the column band of that action on all stacked frames (on top of
low-amplitude noise).  Reward is +1 when the agent's action equals the current target, else 0;
episodes last ``episode_len`` agent steps.  With ``cue_only_first`` the bar is visible only on
the first step after a switch, so acting well requires memory (exercises the LSTM / stored
state / burn-in path).  A greedy agent on random weights scores ~1/A per step; a trained one
approaches 1.

``SyntheticAtariEnv`` is the numpy single-env version with the PongEnv API
(step -> (state float32 (4,84,84)/255, reward, done, info), reset -> state).
``VecSyntheticAtari`` runs E envs on a torch device and writes uint8 frames into a
preallocated (E, 4*84*84) buffer -- the batched GPU actor's input.  On a GPU one env step of all
E envs is ONE kernel (csrc/kernels/env.hip: dynamics + render, counter-hash RNG, graph-safe);
the torch-op version below it serves CPU tensors.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

_VP = ctypes.c_void_p


class EnvArgs(ctypes.Structure):
    """Mirror of ``struct EnvArgs`` (csrc/kernels/env.hip); size checked against the .so."""
    _fields_ = [(n, _VP) for n in ("action", "t", "target", "k", "ep_return", "reward", "done",
                                   "finished", "frames")] + [
        ("seed", ctypes.c_ulonglong)] + [
        (n, ctypes.c_int) for n in ("E", "A", "C", "H", "W", "episode_len", "sw", "cue_only_first")]


class SyntheticAtariEnv:
    def __init__(self, seed: int = 0, episode_len: int = 400, n_actions: int = 6,
                 action_repeat: int = 4, n_stacks: int = 4, switch: int = 8,
                 cue_only_first: bool = False, shape=(84, 84)):
        self.rng = np.random.default_rng(seed)
        self.episode_len = episode_len
        self.n_actions = n_actions
        self.action_repeat = action_repeat
        self.n_stacks = n_stacks
        self.switch = switch
        self.cue_only_first = cue_only_first
        self.h, self.w = shape
        self.t = 0
        self.target = 0

        class _Space:
            def __init__(s, n, rng):
                s.n, s._rng = n, rng

            def sample(s):
                return int(s._rng.integers(s.n))

        self.action_space = _Space(n_actions, self.rng)

    def _frame(self) -> np.ndarray:
        f = self.rng.integers(0, 48, size=(self.n_stacks, self.h, self.w), dtype=np.uint8)
        show = (not self.cue_only_first) or (self.t % self.switch == 0)
        if show:
            band = self.w // self.n_actions
            f[:, :, self.target * band:(self.target + 1) * band] = 220
        return f

    def _obs(self) -> np.ndarray:
        return self._frame().astype(np.float32) / 255.0

    def step(self, action: int):
        reward = 1.0 if int(action) == self.target else 0.0
        self.t += 1
        if self.t % self.switch == 0:
            self.target = int(self.rng.integers(self.n_actions))
        done = self.t >= self.episode_len
        return self._obs(), reward, done, {}

    def reset(self):
        self.t = 0
        self.target = int(self.rng.integers(self.n_actions))
        return self._obs()


class DMLabSynthEnv(SyntheticAtariEnv):
    """96x72 RGB frames (DMLab-30 preset); obs (3*n_stacks, 72, 96)."""

    def __init__(self, seed: int = 0, episode_len: int = 400, n_actions: int = 15, **kw):
        super().__init__(seed=seed, episode_len=episode_len, n_actions=n_actions, n_stacks=3,
                         shape=(72, 96), **kw)


class VecSyntheticAtari:
    """E synthetic envs on a torch device.  ``frames`` (E, C*H*W) uint8 is rewritten in place
    by ``reset_all``/``step`` (the actor's torso kernel reads it directly)."""

    capture_safe = True   # step() is device-only and in place (BatchedActor.capture)

    def __init__(self, n_envs: int, device, seed: int = 0, episode_len: int = 400,
                 n_actions: int = 6, n_stacks: int = 4, switch: int = 8,
                 cue_only_first: bool = False, shape=(84, 84), randomize_start: bool = True):
        self.E, self.A = n_envs, n_actions
        self.device = torch.device(device)
        self.episode_len, self.switch = episode_len, switch
        self.cue_only_first = cue_only_first
        self.C, (self.h, self.w) = n_stacks, shape
        self.g = torch.Generator(device=self.device)
        self.g.manual_seed(seed)
        d = self.device
        self.frames = torch.zeros((n_envs, self.C * self.h * self.w), dtype=torch.uint8, device=d)
        self.t = torch.zeros(n_envs, dtype=torch.int64, device=d)
        self.target = torch.zeros(n_envs, dtype=torch.int64, device=d)
        self.ep_return = torch.zeros(n_envs, dtype=torch.float32, device=d)
        self.randomize_start = randomize_start
        band = self.w // n_actions
        col = torch.arange(self.w, device=d)
        # (A, W) mask of each action's column band
        self._bands = (col[None, :] // band) == torch.arange(n_actions, device=d)[:, None]
        self._bands &= col[None, :] < band * n_actions
        # fused device step (csrc/kernels/env.hip): its state / output buffers are persistent, so
        # a captured actor graph replays it in place
        self._k = torch.zeros(n_envs, dtype=torch.int64, device=d)
        self._reward = torch.zeros(n_envs, dtype=torch.float32, device=d)
        self._done = torch.zeros(n_envs, dtype=torch.bool, device=d)
        self._finished = torch.zeros(n_envs, dtype=torch.float32, device=d)
        self._act = torch.zeros(n_envs, dtype=torch.int64, device=d)
        self._seed = (int(seed) * 0x9E3779B97F4A7C15 + 0x51ED27) & ((1 << 64) - 1)
        self.fused = self.device.type == "cuda"

    def _render(self):
        E = self.E
        noise = torch.randint(0, 48, (E, self.C, self.h, self.w), dtype=torch.uint8,
                              device=self.device, generator=self.g)
        show = torch.ones(E, dtype=torch.bool, device=self.device)
        if self.cue_only_first:
            show = (self.t % self.switch) == 0
        mask = self._bands[self.target] & show[:, None]                  # (E, W)
        noise = torch.where(mask[:, None, None, :], torch.full_like(noise, 220), noise)
        self.frames.copy_(noise.view(E, -1))

    def reset_all(self):
        self.t.zero_()
        if self.randomize_start:  # de-synchronise episode boundaries across envs
            self.t.copy_(torch.randint(0, self.episode_len, (self.E,), device=self.device,
                                       generator=self.g))
        self.target.copy_(torch.randint(0, self.A, (self.E,), device=self.device, generator=self.g))
        self.ep_return.zero_()
        self._render()
        return self.frames

    def _step_fused(self, actions: torch.Tensor):
        from ..ops._lib import check, kernels, stream_handle
        k = kernels()
        if ctypes.sizeof(EnvArgs) != k.r2_env_args_bytes():
            raise RuntimeError("EnvArgs layout differs from csrc/kernels/env.hip")
        act = actions
        if act.dtype != torch.int64 or not act.is_contiguous():
            self._act.copy_(actions.reshape(-1))
            act = self._act
        a = EnvArgs()
        for name, t in (("action", act), ("t", self.t), ("target", self.target), ("k", self._k),
                        ("ep_return", self.ep_return), ("reward", self._reward), ("done", self._done),
                        ("finished", self._finished), ("frames", self.frames)):
            setattr(a, name, t.data_ptr())
        a.seed = self._seed
        a.E, a.A, a.C, a.H, a.W = self.E, self.A, self.C, self.h, self.w
        a.episode_len, a.sw, a.cue_only_first = self.episode_len, self.switch, int(self.cue_only_first)
        check(k.r2_synth_env_step(ctypes.byref(a), _VP(stream_handle())), "synth_env_step")
        return self._reward, self._done, self._finished

    def step(self, actions: torch.Tensor):
        """actions (E,) int on device -> (reward (E,) f32, done (E,) bool, finished_returns).

        Envs whose episode ended are reset in place (their new first frame is rendered)."""
        if self.fused:
            return self._step_fused(actions)
        reward = (actions.long() == self.target).float()
        self.ep_return += reward
        self.t += 1
        sw = (self.t % self.switch) == 0
        new_t = torch.randint(0, self.A, (self.E,), device=self.device, generator=self.g)
        # in place throughout: the batched actor replays this step inside a HIP graph
        self.target.copy_(torch.where(sw, new_t, self.target))
        done = self.t >= self.episode_len
        finished = torch.where(done, self.ep_return, torch.full_like(self.ep_return, float("nan")))
        self.t.masked_fill_(done, 0)
        self.ep_return.masked_fill_(done, 0.0)
        self._render()
        return reward, done, finished
