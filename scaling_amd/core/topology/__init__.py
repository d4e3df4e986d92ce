from .rng_tracker import CudaRNGStateTracker, RngTrackerState
from .topology import Topology, TopologyState, shutdown_distributed
from .topology_config import ActivationCheckpointingType, PipePartitionMethod, TopologyConfig

__all__ = [
    "ActivationCheckpointingType",
    "CudaRNGStateTracker",
    "PipePartitionMethod",
    "RngTrackerState",
    "Topology",
    "TopologyConfig",
    "TopologyState",
    "shutdown_distributed",
]
