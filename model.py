"""Reference module name (``from model import QNet``) -> pytorch_r2d2_amd.models.QNet."""
from pytorch_r2d2_amd.models.qnet import QNet  # noqa: F401
