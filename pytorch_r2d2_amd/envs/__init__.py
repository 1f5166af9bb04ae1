"""Environments.

* ``PongEnv`` -- reference-compatible Atari adapter (``/root/reference/env.py:14-37``): gym
  ``Pong-v0``, gray 84x84, action repeat 4, stack of the 4 frames of the agent step.  Needs
  ``gym`` + ``cv2`` (absent in this image: construction raises a clear error).
* ``SyntheticAtariEnv`` -- deterministic Atari-shaped (4,84,84) uint8 frames, configurable
  episode length and reward; same step/reset API.  Used by tests and benchmarks.
* ``VecSyntheticAtari`` -- the same dynamics for E environments at once on the GPU (frames are
  produced on device, written straight into the actor's input buffer).
* ``CartPoleEnv`` / ``VecCartPole`` -- CartPole-v1 dynamics (numpy / torch vectorised).
* ``DMLabSynthEnv`` -- 96x72 RGB synthetic frames for the DMLab-30 preset.
"""
from .cartpole import CartPoleEnv, VecCartPole
from .pong import PongEnv, preprocess
from .synthetic import DMLabSynthEnv, SyntheticAtariEnv, VecSyntheticAtari


def make_env(cfg, seed: int = 0):
    e = cfg.env
    if e.name == "pong":
        return PongEnv(e.action_repeat, e.n_stacks)
    if e.name == "cartpole":
        return CartPoleEnv(seed=seed, max_steps=e.episode_len)
    if e.name == "dmlab_synth":
        return DMLabSynthEnv(seed=seed, episode_len=e.episode_len, n_actions=e.n_actions,
                             switch=e.switch, cue_only_first=e.cue_only_first)
    return SyntheticAtariEnv(seed=seed, episode_len=e.episode_len, n_actions=e.n_actions,
                             action_repeat=e.action_repeat, n_stacks=e.n_stacks, switch=e.switch,
                             cue_only_first=e.cue_only_first)


__all__ = ["PongEnv", "preprocess", "SyntheticAtariEnv", "VecSyntheticAtari", "CartPoleEnv",
           "VecCartPole", "DMLabSynthEnv", "make_env"]
