"""Op layer: HIP kernels (``torch.ops.dgt``) with plain-PyTorch references for CPU and tests."""
from ._ext import LIB_PATH, available, gpu_available, load, require
from .reference import adam_flat_reference_, tiny_mlp_forward_loss, tiny_mlp_step_reference
from .adam import adam_flat_

__all__ = ["LIB_PATH", "available", "gpu_available", "load", "require", "adam_flat_",
           "adam_flat_reference_", "tiny_mlp_forward_loss", "tiny_mlp_step_reference", "BCEWithLogitsLoss",
           "bce_with_logits", "FusedLinear", "fused_linear", "inject_fused_linear"]
from .loss import BCEWithLogitsLoss, bce_with_logits  # noqa: F401
from .linear import FusedLinear, fused_linear, inject_fused_linear  # noqa: F401
