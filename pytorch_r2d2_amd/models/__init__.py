from .qnet import (QNet, REFERENCE_STATE_DICT_SHAPES, torso_dims, value_rescale,
                   value_rescale_inv)

__all__ = ["QNet", "REFERENCE_STATE_DICT_SHAPES", "torso_dims", "value_rescale",
           "value_rescale_inv"]
