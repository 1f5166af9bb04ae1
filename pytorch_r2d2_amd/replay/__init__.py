from .memory import ReplayMemory
from .nstep import NStepMemory

__all__ = ["ReplayMemory", "NStepMemory"]
