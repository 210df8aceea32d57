"""Flat fused Adam dispatch: HIP kernel on GPU tensors, torch reference on CPU tensors.

Reference: ``train.py:85`` (torch.optim.Adam) stepped at ``train.py:114``; SURVEY K15-K22.
"""
from __future__ import annotations

from typing import Optional

import torch

from ._ext import hot
from .reference import adam_flat_reference_


def adam_flat_(master: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor,
               step: int, lr: float, beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8,
               weight_decay: float = 0.0, adamw: bool = False, grad_scale: float = 1.0,
               grad_scale_dev: Optional[torch.Tensor] = None,
               param_lp: Optional[torch.Tensor] = None, step_dev: Optional[torch.Tensor] = None,
               step_ticket: Optional[torch.Tensor] = None) -> None:
    """One Adam/AdamW step over flat buffers (``master`` fp32 updated in place).

    ``param_lp`` (optional, bf16/fp16) receives the rounded updated parameters;
    ``grad_scale`` and ``grad_scale_dev`` (device scalar, e.g. a clip coefficient) multiply the
    gradient inside the kernel, so DP averaging and clipping cost no extra pass.  ``step_dev`` (a
    device int64 holding this update's 1-based step) replaces ``step`` for HIP-graph replay;
    with ``step_ticket`` (a zeroed device int32 kept beside it) ``step_dev`` holds the steps DONE and
    the launch advances it itself (this update is ``step_dev + 1``): no increment node in a graph.
    """
    if master.is_cuda:
        hot().adam_flat(master, param_lp, grad, exp_avg, exp_avg_sq, float(lr), float(beta1), float(beta2),
                        float(eps), float(weight_decay), bool(adamw), int(step), float(grad_scale),
                        grad_scale_dev, step_dev, step_ticket)
    else:
        if step_dev is not None:
            step = int(step_dev.item())
            if step_ticket is not None:
                step += 1
                step_dev.fill_(step)
        adam_flat_reference_(master, grad, exp_avg, exp_avg_sq, step, lr, beta1, beta2, eps, weight_decay,
                             adamw, grad_scale, grad_scale_dev, param_lp)
