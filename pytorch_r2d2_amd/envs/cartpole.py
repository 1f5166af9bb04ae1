"""CartPole-v1 dynamics (no gym in this image): numpy single env + torch vectorised env.

Physics constants and termination follow the classic Barto/Sutton cart-pole as in gym's
CartPole-v1 (gravity 9.8, masscart 1.0, masspole 0.1, length 0.5, force 10, tau 0.02, Euler
integration, |x| > 2.4 or |theta| > 12 deg terminates, 500-step limit, reward 1 per step).
"""
from __future__ import annotations

import math

import numpy as np
import torch

G, MC, MP, LEN, FORCE, TAU = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
TOTAL = MC + MP
PML = MP * LEN
TH_LIM = 12 * 2 * math.pi / 360
X_LIM = 2.4


def _dyn(x, xd, th, thd, force, cos, sin):
    temp = (force + PML * thd * thd * sin) / TOTAL
    thacc = (G * sin - cos * temp) / (LEN * (4.0 / 3.0 - MP * cos * cos / TOTAL))
    xacc = temp - PML * thacc * cos / TOTAL
    return x + TAU * xd, xd + TAU * xacc, th + TAU * thd, thd + TAU * thacc


class CartPoleEnv:
    def __init__(self, seed: int = 0, max_steps: int = 500):
        self.rng = np.random.default_rng(seed)
        self.max_steps = max_steps
        self.state = np.zeros(4, dtype=np.float32)
        self.t = 0

        class _Space:
            n = 2

            def __init__(s, rng):
                s._rng = rng

            def sample(s):
                return int(s._rng.integers(2))

        self.action_space = _Space(self.rng)

    def reset(self):
        self.state = self.rng.uniform(-0.05, 0.05, size=4).astype(np.float32)
        self.t = 0
        return self.state.copy()

    def step(self, action: int):
        x, xd, th, thd = (float(v) for v in self.state)
        force = FORCE if int(action) == 1 else -FORCE
        x, xd, th, thd = _dyn(x, xd, th, thd, force, math.cos(th), math.sin(th))
        self.state = np.array([x, xd, th, thd], dtype=np.float32)
        self.t += 1
        done = abs(x) > X_LIM or abs(th) > TH_LIM or self.t >= self.max_steps
        return self.state.copy(), 1.0, done, {}


class VecCartPole:
    def __init__(self, n_envs: int, device="cpu", seed: int = 0, max_steps: int = 500):
        self.E = n_envs
        self.device = torch.device(device)
        self.g = torch.Generator(device=self.device)
        self.g.manual_seed(seed)
        self.max_steps = max_steps
        self.state = torch.zeros(n_envs, 4, device=self.device)
        self.t = torch.zeros(n_envs, dtype=torch.int64, device=self.device)
        self.ep_return = torch.zeros(n_envs, device=self.device)

    def _init(self, n):
        return (torch.rand(n, 4, device=self.device, generator=self.g) - 0.5) * 0.1

    def reset_all(self):
        self.state = self._init(self.E)
        self.t.zero_()
        self.ep_return.zero_()
        return self.state

    def step(self, actions: torch.Tensor):
        x, xd, th, thd = self.state.unbind(1)
        force = torch.where(actions.long() == 1, FORCE, -FORCE).float()
        x, xd, th, thd = _dyn(x, xd, th, thd, force, torch.cos(th), torch.sin(th))
        self.state = torch.stack([x, xd, th, thd], 1)
        self.t += 1
        reward = torch.ones(self.E, device=self.device)
        self.ep_return += reward
        done = (x.abs() > X_LIM) | (th.abs() > TH_LIM) | (self.t >= self.max_steps)
        finished = torch.where(done, self.ep_return, torch.full_like(self.ep_return, float("nan")))
        fresh = self._init(self.E)
        self.state = torch.where(done[:, None], fresh, self.state)
        self.t = torch.where(done, torch.zeros_like(self.t), self.t)
        self.ep_return = torch.where(done, torch.zeros_like(self.ep_return), self.ep_return)
        return reward, done, finished
