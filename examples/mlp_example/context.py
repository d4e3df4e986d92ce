from scaling_amd.core import BaseContext, Topology

from .config import MLPConfig


class MLPContext(BaseContext):
    config: MLPConfig

    def __init__(self, config: MLPConfig, topology: Topology):
        super().__init__(config=config, topology=topology)
