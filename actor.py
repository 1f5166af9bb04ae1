"""Reference module name (``from actor import actor_process``) -> pytorch_r2d2_amd.actor."""
from pytorch_r2d2_amd.actor import Actor, actor_process  # noqa: F401
