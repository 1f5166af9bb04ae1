"""Reference module name (``from replay_memory import NStepMemory, ReplayMemory``)."""
from pytorch_r2d2_amd.replay.memory import ReplayMemory  # noqa: F401
from pytorch_r2d2_amd.replay.nstep import NStepMemory  # noqa: F401
