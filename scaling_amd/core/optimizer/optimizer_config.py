from pydantic import Field

from ..config import BaseConfig
from .loss_scaler_config import LossScalerConfig


class OptimizerConfig(BaseConfig):
    method: str = Field("adamw", description="Which optimization method to use.")
    beta1: float = Field(0.9, description="AdamW beta1")
    beta2: float = Field(0.95, description="AdamW beta2")
    eps: float = Field(1e-8, description="AdamW epsilon")
    gradient_clipping: float = Field(1.0, description="clip global l2 grads to this value, deactivate if 0.0", ge=0.0)
    allreduce_bucket_size: int = Field(500000000, description="upper bound of elements per gradient bucket", gt=0)
    loss_scaler: LossScalerConfig = Field(LossScalerConfig(), description="Configuration of the loss scaler")
    zero: bool = Field(False, description="enable ZeRO stage 1 (optimizer state sharded over data parallel)")
    zero_save_static: bool = Field(False, description="save per-rank optimizer files instead of merged per-layer files")
    debug_log: bool = Field(False)
    # --- MI355X-native additions (optional) ---
    grad_bucket_numel: int = Field(
        2**26,
        description="elements per gradient communication bucket (reduce-scatter / all-gather granularity); "
        "buckets are launched on a side stream as soon as their grads are final (overlap with backward)",
        gt=0,
    )
    grad_reduce_dtype: str = Field(
        "float32", description="dtype of the data-parallel gradient reduction ('float32' as the reference, or 'bfloat16')"
    )
    overlap_grad_reduce: bool = Field(True, description="overlap the data-parallel gradient reduction with backward")
    overlap_optimizer_step: bool = Field(
        True,
        description="run the AdamW update (and the ZeRO all-gather) bucket by bucket on a side stream; the next "
        "forward waits per layer for its buckets, the next backward for the gradient zeroing (GPU only)",
    )
    lazy_grad_zeroing: bool = Field(
        False,
        description="defer each parameter's gradient zeroing to its first gradient write of the next step (the "
        "GEMM-fused weight gradient then writes with beta = 0): no full-buffer memset per step.  Requires that "
        "gradients are produced only by backward passes (code that writes .grad directly must leave it off)",
    )
    overlap_param_gather: bool = Field(
        True,
        description="ZeRO: all-gather updated parameters bucket by bucket on a side stream and let each pipeline "
        "layer's next forward wait only for its own buckets (overlaps the all-gather with the next step)",
    )
