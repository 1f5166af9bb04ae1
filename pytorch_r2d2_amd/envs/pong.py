"""Reference-compatible Pong adapter (``/root/reference/env.py``).

Behaviour kept from the reference: gray 84x84 uint8 frames (env.py:8-11), action repeat 4
summing reward and stopping on ``done`` (env.py:21-31), a 4-deep frame deque fed one frame per
raw step so each returned (4,84,84) stack holds the frames of this agent step (env.py:18,26,30),
float32/255 output, and 1-4 random-action agent steps on reset (env.py:33-37).

Fixed: both the old (4-tuple step, obs reset) and new (5-tuple step, (obs, info) reset) gym
APIs are accepted (Q15).  ``gym``/``cv2`` are optional imports; without them construction
raises ImportError with an explanation (use ``SyntheticAtariEnv``).
"""
from __future__ import annotations

from collections import deque

import numpy as np


def _resize_gray(frame: np.ndarray) -> np.ndarray:
    try:
        import cv2  # type: ignore
        return cv2.resize(cv2.cvtColor(frame, cv2.COLOR_RGB2GRAY), (84, 84))
    except ImportError:
        return _resize_gray_area(frame)


def _resize_gray_area(frame: np.ndarray) -> np.ndarray:
    """Dependency-free fallback: ITU-R 601 luma + area-average resize to 84x84, vectorised over an
    integral image (every output cell is the mean of rows [ys[i], ye[i]) x cols [xs[j], xe[j]))."""
    g = frame[..., 0] * 0.299 + frame[..., 1] * 0.587 + frame[..., 2] * 0.114
    h, w = g.shape
    ys = (np.arange(85) * h / 84).astype(int)
    xs = (np.arange(85) * w / 84).astype(int)
    y0, y1 = ys[:84], np.maximum(ys[1:], ys[:84] + 1)
    x0, x1 = xs[:84], np.maximum(xs[1:], xs[:84] + 1)
    S = np.zeros((h + 1, w + 1), dtype=np.float64)
    S[1:, 1:] = g.cumsum(0).cumsum(1)
    tot = S[y1][:, x1] - S[y0][:, x1] - S[y1][:, x0] + S[y0][:, x0]
    return (tot / ((y1 - y0)[:, None] * (x1 - x0)[None, :])).astype(np.float32)


def preprocess(frame: np.ndarray) -> np.ndarray:
    """RGB (210,160,3) -> uint8 (1,84,84) (env.py:8-11)."""
    return np.uint8(_resize_gray(frame)).reshape(1, 84, 84)


class PongEnv:
    def __init__(self, action_repeat: int = 4, n_stacks: int = 4, env_id: str = "Pong-v0",
                 gym_env=None):
        self.action_repeat = action_repeat
        self.n_stacks = n_stacks
        self.frame_queue = deque(maxlen=self.n_stacks)
        if gym_env is None:
            try:
                import gym  # type: ignore
            except ImportError as e:  # pragma: no cover - depends on image
                raise ImportError("PongEnv needs `gym` with the Atari ROMs (not installed in this "
                                  "image); use pytorch_r2d2_amd.envs.SyntheticAtariEnv") from e
            gym_env = gym.make(env_id)
        self.env = gym_env
        self.action_space = getattr(gym_env, "action_space", None)

    def _raw_step(self, action):
        out = self.env.step(action)
        if len(out) == 5:
            frame, reward, term, trunc, info = out
            return frame, reward, bool(term or trunc), info
        return out

    def step(self, action):
        total_reward = 0.0
        done, info = False, {}
        for _ in range(self.action_repeat):
            frame, reward, done, info = self._raw_step(action)
            self.frame_queue.append(preprocess(frame))
            total_reward += reward
            if done:
                break
        while len(self.frame_queue) < self.n_stacks:
            self.frame_queue.appendleft(self.frame_queue[0])
        state = np.concatenate(list(self.frame_queue)).astype(np.float32) / 255.0
        return state, total_reward, done, info

    def reset(self):
        out = self.env.reset()
        if isinstance(out, tuple) and len(out) == 2 and isinstance(out[1], dict):
            out = out[0]
        state = None
        for _ in range(np.random.randint(1, 5)):
            a = self.action_space.sample() if self.action_space is not None else 0
            state, _, _, _ = self.step(a)
        return state
