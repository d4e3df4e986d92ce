"""scaling_amd — MI355X-native (gfx950) 3D-parallel training framework.

Public API mirrors Aleph Alpha's Scaling library (``scaling.core`` / ``scaling.transformer``):
import ``scaling_amd.core`` / ``scaling_amd.transformer``, or the ``scaling`` compatibility alias.
Hot ops are hand-written HIP kernels for CDNA4 (``scaling_amd.ops``), communication is RCCL over
xGMI via torch.distributed (``scaling_amd.parallel``).
"""
__version__ = "0.1.0"
