"""pytorch_r2d2_amd -- MI355X-native R2D2 (Recurrent Replay Distributed DQN).

Feature parity with LiXirong/pytorch-r2d2 re-designed for AMD Instinct MI355X:
HIP/CDNA4 kernels for the learner and actor hot paths, HBM-resident prioritized sequence replay,
RCCL-over-xGMI data parallelism, and a native C++ host runtime.
"""
from .config import R2D2Config, get_config  # noqa: F401

__version__ = "0.1.0"
