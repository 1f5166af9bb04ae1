from .checkpoint import (load_full_checkpoint, load_reference_checkpoint, save_full_checkpoint,
                         save_reference_checkpoint)
from .faults import faults, set_faults
from .metrics import MetricsLogger, RateMeter, read_jsonl
from .profiling import PhaseTimer, roctx_mark, roctx_range

__all__ = ["load_full_checkpoint", "load_reference_checkpoint", "save_full_checkpoint",
           "save_reference_checkpoint", "faults", "set_faults", "MetricsLogger", "RateMeter",
           "read_jsonl", "PhaseTimer", "roctx_range", "roctx_mark"]
