from .dist import DistInfo, barrier, init_distributed, shutdown
from .grad_sync import GradSync, allreduce_mean_
from .sharded_replay import gather_stats, global_is_params, local_stats
from .trajectory import ShmTrajectoryReader, ShmTrajectoryWriter, pack_rows, unpack_rows
from .weights import SharedDictWeights, WeightPublisher

__all__ = ["DistInfo", "barrier", "init_distributed", "shutdown", "GradSync", "allreduce_mean_",
           "gather_stats", "global_is_params", "local_stats", "ShmTrajectoryReader",
           "ShmTrajectoryWriter", "pack_rows", "unpack_rows", "SharedDictWeights",
           "WeightPublisher"]
