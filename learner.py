"""Reference module name (``from learner import learner_process``) -> pytorch_r2d2_amd.learner."""
from pytorch_r2d2_amd.learner import Learner, learner_process  # noqa: F401
