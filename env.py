"""Reference module name (``from env import PongEnv``) -> pytorch_r2d2_amd.envs."""
from pytorch_r2d2_amd.envs.pong import PongEnv, preprocess  # noqa: F401
