"""Plain-PyTorch reference implementations of the fused ops.

These run anywhere (CPU in the test container, GPU as numerics oracles) and define the exact op
order the HIP kernels reproduce:

* ``adam_flat_reference_`` — ``torch.optim.Adam``'s foreach update (``torch/optim/adam.py``
  ``_multi_tensor_adam``: lerp_, mul_, addcmul_, sqrt, div_, add_, addcdiv_) on flat buffers,
  with the bias corrections formed in double on the host exactly as torch does.
* ``tiny_mlp_step_reference`` — one step of the reference model (``train.py:107-113``):
  Linear -> ReLU -> Linear -> BCEWithLogits(mean) and its analytic backward into a flat gradient.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch


def adam_flat_reference_(master: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor,
                         exp_avg_sq: torch.Tensor, step: int, lr: float, beta1: float = 0.9,
                         beta2: float = 0.999, eps: float = 1e-8, weight_decay: float = 0.0,
                         adamw: bool = False, grad_scale: float = 1.0,
                         grad_scale_dev: Optional[torch.Tensor] = None,
                         param_lp: Optional[torch.Tensor] = None) -> None:
    g = grad.float()
    if grad_scale != 1.0:
        g = g * grad_scale
    if grad_scale_dev is not None:
        g = g * grad_scale_dev.float()
    if weight_decay != 0.0:
        if adamw:
            master.mul_(1 - lr * weight_decay)
        else:
            g = g.add(master, alpha=weight_decay)
    exp_avg.lerp_(g, 1 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    step_size = lr / bc1
    denom = (exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(eps)
    master.addcdiv_(exp_avg, denom, value=-step_size)
    if param_lp is not None:
        param_lp.copy_(master)


def tiny_mlp_forward_loss(flat: torch.Tensor, x: torch.Tensor, y: torch.Tensor, n_features: int,
                          hidden: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    F, H = n_features, hidden
    w1 = flat[: H * F].view(H, F)
    b1 = flat[H * F: H * F + H]
    w2 = flat[H * F + H: H * F + 2 * H]
    b2 = flat[H * F + 2 * H]
    pre = x @ w1.t() + b1
    h = torch.relu(pre)
    z = h @ w2 + b2
    loss = torch.nn.functional.binary_cross_entropy_with_logits(z, y.view(-1))
    return loss, h, z


def tiny_mlp_step_reference(flat: torch.Tensor, x: torch.Tensor, y: torch.Tensor, n_features: int,
                            hidden: int, grad_out: Optional[torch.Tensor] = None) -> Tuple[float, torch.Tensor]:
    """Return (mean loss, flat gradient) for one minibatch; gradient has ``flat``'s length."""
    F, H = n_features, hidden
    loss, h, z = tiny_mlp_forward_loss(flat, x, y, F, H)
    B = x.shape[0]
    w2 = flat[H * F + H: H * F + 2 * H]
    dz = (torch.sigmoid(z) - y.view(-1)) / B
    g = torch.zeros_like(flat) if grad_out is None else grad_out.zero_()
    g[H * F + H: H * F + 2 * H] = dz @ h
    g[H * F + 2 * H] = dz.sum()
    dh = torch.outer(dz, w2) * (h > 0)
    g[H * F: H * F + H] = dh.sum(0)
    g[: H * F] = (dh.t() @ x).reshape(-1)
    return float(loss), g
