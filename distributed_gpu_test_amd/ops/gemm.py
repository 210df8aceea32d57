"""bf16 MFMA GEMM + MLP helper ops (``csrc/gemm.hip``) with plain-PyTorch references.

Reference: the Linear layers of ``train.py:29-33`` (forward ``train.py:107``, backward ``train.py:113``), scaled up.

``gemm_nt`` computes ``C = alpha * A @ B.T`` (A[M,K], B[N,K], both bf16, fp32 accumulation) with
optional fused epilogue: ``+ bias``, ``relu``, ``* 1[mask > 0]``, a transposed bf16 copy ``CT``,
fp32 output / accumulation.  On GPU tensors it runs the HIP kernel (and raises if the extension
is missing); on CPU tensors it runs the reference, which is also the numerics oracle in tests.
"""
from __future__ import annotations

from typing import Optional

import torch

from ._ext import require

EPI_BIAS, EPI_RELU, EPI_MASK, EPI_STORE_T, EPI_OUT_F32, EPI_ACCUMULATE, EPI_B_KN = 1, 2, 4, 8, 16, 32, 64


def gemm_nt_reference(A, B, C=None, CT=None, bias=None, mask=None, relu=False, out_f32=False,
                      accumulate=False, alpha=1.0, b_kn=False):
    r = (A.float() @ (B.float() if b_kn else B.float().t())) * alpha
    if bias is not None:
        r = r + bias.float()
    if relu:
        r = torch.relu(r)
    if mask is not None:
        r = torch.where(mask.float() > 0, r, torch.zeros_like(r))
    if C is not None:
        if out_f32 and accumulate:
            C.add_(r)
        else:
            C.copy_(r.to(C.dtype))
    if CT is not None:
        CT.copy_(r.t().to(CT.dtype))
    return r


def gemm_nt(A: torch.Tensor, B: torch.Tensor, C: Optional[torch.Tensor] = None, CT: Optional[torch.Tensor] = None,
            bias: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None, relu: bool = False,
            out_f32: bool = False, accumulate: bool = False, alpha: float = 1.0, variant: int = 0,
            b_kn: bool = False) -> None:
    """variant: 0 = pick the kernel by shape, 1 = 128x128 tiles 2-stage, 2 = 256x256 8-phase pipeline,
    3 = 128x128 tiles 4-stage, 4 = 128x128 tiles 4-stage with 8 waves, 5 = 256x128 tiles with K
    split over two blocks that meet through a per-tile counter (the M = 1024 MLP products),
    7 = 128x128 tiles, 8 waves, 2 stages of BK = 128 (K % 128 == 0; one block per CU),
    8 = 128x128 tiles, 8 waves, 5 stages of BK = 64 with one barrier per two K-tiles (K % 128 == 0).

    ``b_kn=True``: B is given as ``[K, N]`` (N contiguous) and ``C = alpha * A @ B`` — the operand is
    staged as it lies and read with transposed LDS reads (128x128 kernels only)."""
    if not A.is_cuda:
        gemm_nt_reference(A, B, C, CT, bias, mask, relu, out_f32, accumulate, alpha, b_kn)
        return
    epi = ((EPI_BIAS if bias is not None else 0) | (EPI_RELU if relu else 0) | (EPI_MASK if mask is not None else 0)
           | (EPI_STORE_T if CT is not None else 0) | (EPI_OUT_F32 if out_f32 else 0)
           | (EPI_ACCUMULATE if accumulate else 0) | (EPI_B_KN if b_kn else 0))
    M, N = A.shape[0], B.shape[1] if b_kn else B.shape[0]
    slab, flags = _sk_workspace(A.device, M, N) if variant == 5 and not out_f32 else (None, None)
    require().gemm_nt(A, B, C, CT, bias, mask, epi, float(alpha), int(variant), slab, flags)


_SK: dict = {}


def _sk_workspace(device: torch.device, M: int, N: int):
    """Workspace of the split-K kernel (variant 5): fp32 partial tiles + zeroed per-tile flags that
    the kernel re-arms.  One per (device, stream): launches sharing it are stream-ordered."""
    if M % 256 or N % 128 or ((M // 256) * (N // 128)) % 8:
        return None, None
    tiles = (M // 256) * (N // 128)
    key = (device.index, torch.cuda.current_stream(device).cuda_stream)
    ws = _SK.get(key)
    if ws is None or ws[1].numel() < 2 * tiles:
        ws = (torch.empty(tiles * 256 * 128, dtype=torch.float32, device=device),
              torch.zeros(2 * tiles, dtype=torch.int32, device=device))
        _SK[key] = ws
    return ws


def gemm_nt_adam_(A: torch.Tensor, B: torch.Tensor, master: torch.Tensor, exp_avg: torch.Tensor,
                  exp_avg_sq: torch.Tensor, param_lp: torch.Tensor, step: int, lr: float, beta1: float, beta2: float,
                  eps: float, weight_decay: float = 0.0, adamw: bool = False, grad_scale: float = 1.0,
                  variant: int = 0) -> None:
    """Weight gradient ``grad_scale * A @ B.T`` ([M, N], never materialised) consumed in place by
    Adam: updates the fp32 ``master`` / ``exp_avg`` / ``exp_avg_sq`` ([M, N]) and writes the bf16
    compute copy ``param_lp``.  One launch instead of wgrad GEMM + gradient store + flat Adam.
    variant as ``gemm_nt`` (0-4, 7, 8), or 6: persistent blocks whose MFMA waves hand each finished tile
    to Adam waves that update it while the next tile computes (K = 1024 only)."""
    if not A.is_cuda:
        from .reference import adam_flat_reference_
        g = (A.float() @ B.float().t()).reshape(-1)
        p, m, v = master.view(-1), exp_avg.view(-1), exp_avg_sq.view(-1)
        adam_flat_reference_(p, g, m, v, step, lr, beta1, beta2, eps, weight_decay, adamw, grad_scale=grad_scale)
        param_lp.copy_(master.to(param_lp.dtype))
        return
    require().gemm_nt_adam(A, B, master, exp_avg, exp_avg_sq, param_lp, int(step), float(lr), float(beta1),
                           float(beta2), float(eps), float(weight_decay), bool(adamw), float(grad_scale), int(variant))


def transpose_bf16(inp: torch.Tensor, out: torch.Tensor) -> None:
    if inp.is_cuda:
        require().transpose_bf16(inp, out)
    else:
        out.copy_(inp.t())


def rowsum_bf16(inp: torch.Tensor, out: torch.Tensor, accumulate: bool = False) -> None:
    if inp.is_cuda:
        require().rowsum_bf16(inp, out, accumulate)
    else:
        s = inp.float().sum(1)
        out.add_(s) if accumulate else out.copy_(s)


def mlp_head(a, w, b0, y, dz, dw, db, loss_acc, g, gT) -> None:
    """Linear(D,1) + BCE-with-logits (mean) forward and backward; dw, db are overwritten with the
    head's gradients, loss_acc accumulates the mean loss."""
    if a.is_cuda:
        require().mlp_head(a, w, b0, y, dz, dw, db, loss_acc, g, gT)
        return
    af = a.float()
    z = af @ w + b0
    loss = torch.nn.functional.binary_cross_entropy_with_logits(z, y)
    d = (torch.sigmoid(z) - y) / a.shape[0]
    dz.copy_(d)
    dw.copy_(d @ af)
    db.copy_(d.sum())
    loss_acc.add_(float(loss))
    gg = torch.outer(d, w) * (af > 0)
    g.copy_(gg.to(g.dtype))
    gT.copy_(gg.t().to(gT.dtype))
