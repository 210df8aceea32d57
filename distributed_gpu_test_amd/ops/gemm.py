"""bf16 MFMA GEMM + MLP helper ops (``csrc/gemm.hip``) with plain-PyTorch references.

Reference: the Linear layers of ``train.py:29-33`` (forward ``train.py:107``, backward ``train.py:113``), scaled up.

``gemm_nt`` computes ``C = alpha * A @ B.T`` (A[M,K], B[N,K], both bf16, fp32 accumulation) with
optional fused epilogue: ``+ bias``, ``relu``, ``* 1[mask > 0]``, a transposed bf16 copy ``CT``,
fp32 output / accumulation.  On GPU tensors it runs the HIP kernel (and raises if the extension
is missing); on CPU tensors it runs the reference, which is also the numerics oracle in tests.
"""
from __future__ import annotations

from typing import Optional

import os

import torch

from ._ext import require

EPI_BIAS, EPI_RELU, EPI_MASK, EPI_STORE_T, EPI_OUT_F32, EPI_ACCUMULATE, EPI_B_KN = 1, 2, 4, 8, 16, 32, 64


def gemm_nt_reference(A, B, C=None, CT=None, bias=None, mask=None, relu=False, out_f32=False,
                      accumulate=False, alpha=1.0, b_kn=False, colsum=None):
    r = (A.float() @ (B.float() if b_kn else B.float().t())) * alpha
    if bias is not None:
        r = r + bias.float()
    if relu:
        r = torch.relu(r)
    if mask is not None:
        r = torch.where(mask.float() > 0, r, torch.zeros_like(r))
    if colsum is not None:  # per-128-row-tile column sums of the bf16-rounded output
        colsum.copy_(r.to(torch.bfloat16).float().view(r.shape[0] // 128, 128, r.shape[1]).sum(1))
    if C is not None:
        if accumulate:
            C.copy_((C.float() + r).to(C.dtype))
        else:
            C.copy_(r.to(C.dtype))
    if CT is not None:
        CT.copy_(r.t().to(CT.dtype))
    return r


_ENV_VARIANT = int(os.environ.get("DGT_GEMM_VARIANT", "0") or 0)


def gemm_nt(A: torch.Tensor, B: torch.Tensor, C: Optional[torch.Tensor] = None, CT: Optional[torch.Tensor] = None,
            bias: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None, relu: bool = False,
            out_f32: bool = False, accumulate: bool = False, alpha: float = 1.0, variant: int = 0,
            b_kn: bool = False, colsum: Optional[torch.Tensor] = None) -> None:
    """variant: 0 = pick the kernel by shape, 1 = 128x128 tiles 2-stage (2 blocks per CU),
    2 = 256x256 8-phase pipeline (variant 8's bitwise oracle), 3 = variant 4 with front-loaded LDS
    fragment reads,
    4 = 128x128 tiles 4-stage with 8 waves (1 block per CU; variant 3's bitwise oracle),
    5 = software-pipelined fragment reads (the next K-tile's fragments read during this one's MFMAs,
    five LDS stages; K % 128 == 0, else 3) -- the shape rule's choice for the ``b_kn`` dgrad,
    6 / 7 = register prefetch (2 / 4 K-tiles of operands in flight in VGPRs, two LDS stages; NT
    forward-type products, bit-identical to 3; other products keep the shape rule),
    8 = the 256x256 kernel with cross-phase fragment prefetch (phase P's MFMAs overlap the LDS
    reads of phase P + 1; bit-identical to 2) -- the kernel the shape rule runs for >= 200 tiles of
    256x256,
    9 = 256x128 tiles with K split in two halves that meet in-launch (per 128-row half: one block
    publishes its fp32 partial, the other finishes; deterministic; M % 256 == 0, N % 128 == 0, K % 128 == 0, a multiple of 8 tiles, bf16 epilogues,
    ``b_kn`` and ``colsum`` included) -- opt-in: ``DGT_GEMM_SK=1`` makes the shape rule use it for
    one-wave NT grids with K >= 2048; on the MLP's M = 1024 products it is no faster than 3 / 5
    (``profiles/r6_gemm_m1024_splitk.jsonl``),
    10 = the 128x128 kernel with K split 2 / 4 / 8 ways for grids of at most 128 tiles (small M): the
    slices meet in-launch, the last to arrive sums them in slice order (deterministic) -- the shape
    rule's choice there (``DGT_GEMM_SKN=0`` turns it off),
    11 = the 256x256 kernel with K split in two (NT, staged bf16 epilogues without column sums; the
    second block to finish adds the first's fp32 partial): the shape rule's choice for 100-128 tiles
    of 256x256, e.g. 1024 x 8192 (``profiles/r6_gemm_wide_8192.jsonl``).
    ``DGT_GEMM_VARIANT`` (A/B runs) replaces variant 0 for grids of at most 256 tiles (the shapes
    the shape rule gives to the 128x128 kernels).

    ``b_kn=True``: B is given as ``[K, N]`` (N contiguous) and ``C = alpha * A @ B`` — the operand is
    staged as it lies and read with transposed LDS reads (128x128 and split-K kernels).  ``accumulate``
    adds into C (fp32, or bf16 summed in fp32 and rounded once).

    ``colsum`` (fp32 ``[M // 128, N]``, the ``[K, N]`` dgrad with ``mask`` and ``CT`` only): each
    128-row tile's column sums of the bf16 output -- the next layer's bias-gradient partials, formed
    in the epilogue from the values already staged for ``CT`` (``partials_reduce_multi`` finishes
    them)."""
    if not A.is_cuda:
        gemm_nt_reference(A, B, C, CT, bias, mask, relu, out_f32, accumulate, alpha, b_kn, colsum)
        return
    epi = ((EPI_BIAS if bias is not None else 0) | (EPI_RELU if relu else 0) | (EPI_MASK if mask is not None else 0)
           | (EPI_STORE_T if CT is not None else 0) | (EPI_OUT_F32 if out_f32 else 0)
           | (EPI_ACCUMULATE if accumulate else 0) | (EPI_B_KN if b_kn else 0))
    if variant == 0 and _ENV_VARIANT and (A.shape[0] // 128) * ((B.shape[1] if b_kn else B.shape[0]) // 128) <= 256:
        variant = _ENV_VARIANT
    require().gemm_nt(A, B, C, CT, bias, mask, epi, float(alpha), int(variant), colsum)


def partials_reduce_multi(pairs, adam=None) -> None:
    """For every ``(part [tiles, n], out [n])`` pair (part fp32, out fp32 or bf16): ``out =
    part.sum(0)``, the tiles added in order -- all pairs in ONE launch (at most 8).  A pair may carry a
    third element ``accumulate``: ``out += part.sum(0)`` (a bf16 out: the sum in fp32, rounded once).
    ``adam`` = ``(grads, master, exp_avg,
    exp_avg_sq, step, lr, beta1, beta2, eps, weight_decay, adamw, grad_scale)``: the outs are views of
    ``grads`` and the same launch applies Adam to their elements of master / exp_avg / exp_avg_sq
    (adam_flat's arithmetic: the same bits as a separate adam_flat over the region)."""
    pairs = [(q[0], q[1], bool(q[2]) if len(q) > 2 else False) for q in pairs]
    parts, outs = [q[0] for q in pairs], [q[1] for q in pairs]
    acc_flags = [int(q[2]) for q in pairs] if any(q[2] for q in pairs) else None
    if parts[0].is_cuda:
        if adam is None:
            require().partials_reduce_multi(parts, outs, accumulate=acc_flags)
        else:
            g, p_, m, v, step, lr, b1, b2, eps, wd, adamw, scale = adam
            require().partials_reduce_multi(parts, outs, g, p_, m, v, int(step), float(lr), float(b1), float(b2),
                                            float(eps), float(wd), bool(adamw), float(scale), acc_flags)
        return
    for p, o, accumulate in pairs:
        acc = torch.zeros_like(p[0])
        for t in range(p.shape[0]):
            acc += p[t]
        if accumulate:  # the kernel's order: the tiles' sum, then added to the out
            acc = o.float().reshape(-1) + acc
        o.copy_(acc.view(o.shape).to(o.dtype))
    if adam is not None:
        from .reference import adam_flat_reference_
        g, p_, m, v, step, lr, b1, b2, eps, wd, adamw, scale = adam
        for _, o, _ in pairs:
            off = (o.data_ptr() - g.data_ptr()) // 4
            sl = slice(off, off + o.numel())
            adam_flat_reference_(p_[sl], g[sl], m[sl], v[sl], step, lr, b1, b2, eps, wd, adamw, grad_scale=scale)


def gemm_nt_adam_(A: torch.Tensor, B: torch.Tensor, master: torch.Tensor, exp_avg: torch.Tensor,
                  exp_avg_sq: torch.Tensor, param_lp: torch.Tensor, step: int, lr: float, beta1: float, beta2: float,
                  eps: float, weight_decay: float = 0.0, adamw: bool = False, grad_scale: float = 1.0,
                  variant: int = 0) -> None:
    """Weight gradient ``grad_scale * A @ B.T`` ([M, N], never materialised) consumed in place by
    Adam: updates the fp32 ``master`` / ``exp_avg`` / ``exp_avg_sq`` ([M, N]) and writes the bf16
    compute copy ``param_lp``.  One launch instead of wgrad GEMM + gradient store + flat Adam.
    variant as ``gemm_nt``."""
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
    """out (fp32 or bf16) [rows] (+)= row sums of a bf16 [rows, cols] matrix (summed in fp32)."""
    if inp.is_cuda:
        require().rowsum_bf16(inp, out, accumulate)
    else:
        s = inp.float().sum(1)
        out.copy_((out.float() + s).to(out.dtype) if accumulate else s.to(out.dtype))


def skinny_fwd_bf16(a: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], z: torch.Tensor) -> None:
    """Head Linear(K, N <= 4) in bf16: z[M, N] = a . w^T + b (fp32 accumulation, csrc/head.hip)."""
    if a.is_cuda:
        require().skinny_fwd_bf16(a, w, b, z)
        return
    r = a.float() @ w.float().t()
    if b is not None:
        r = r + b.float()
    z.copy_(r.reshape(z.shape).to(z.dtype))


def skinny_bwd_bf16(dz: torch.Tensor, a: torch.Tensor, w: torch.Tensor, mask: bool, g: torch.Tensor,
                    gT: Optional[torch.Tensor], dw: torch.Tensor, db: torch.Tensor, accumulate: bool = True,
                    bias_part: Optional[torch.Tensor] = None, dw_part: Optional[torch.Tensor] = None) -> None:
    """Its backward: g = (dz . w) * 1[a > 0] (if mask) and g^T (bf16); dw [N, K] and db [N] (both fp32
    or both bf16) receive dz^T . a and the column sums of dz: added (``accumulate``) or stored.
    ``bias_part`` (fp32 ``[M // 64, K]``): the per-64-row-tile column sums of the bf16 g (the layer
    below's bias-gradient partials, for ``partials_reduce_multi``).  ``dw_part`` (fp32 ``[M // 64, N * K]``):
    dw's per-64-row-tile partials are left there for the caller to reduce, and dw is not written."""
    if a.is_cuda:
        require().skinny_bwd_bf16(dz, a, w, mask, g, gT, dw, db, bool(accumulate), bias_part, dw_part)
        return
    d = dz.float().reshape(a.shape[0], w.shape[0])
    gg = d @ w.float()
    if mask:
        gg = gg * (a.float() > 0)
    g.copy_(gg.to(g.dtype))
    if bias_part is not None:
        bias_part.copy_(g.float().view(-1, 64, g.shape[1]).sum(1))
    if gT is not None:
        gT.copy_(gg.t().to(gT.dtype))
    if dw_part is not None:
        t = a.shape[0] // 64
        dw_part.copy_(torch.einsum("trn,trk->tnk", d.view(t, 64, -1), a.float().view(t, 64, -1)).reshape(t, -1))
        db.copy_(((db.float() + d.sum(0)) if accumulate else d.sum(0)).to(db.dtype))
        return
    if accumulate:
        dw.copy_((dw.float() + d.t() @ a.float()).to(dw.dtype))
        db.copy_((db.float() + d.sum(0)).to(db.dtype))
    else:
        dw.copy_((d.t() @ a.float()).to(dw.dtype))
        db.copy_(d.sum(0).to(db.dtype))


def mlp_head(a, w, b0, y, dz, dw, db, loss_acc, g, gT, dw_part=None, bias_part=None) -> None:
    """Linear(D,1) + BCE-with-logits (mean) forward and backward; dw, db are overwritten with the
    head's gradients, loss_acc accumulates the mean loss.  ``dw_part`` (fp32 ``[B // 64, D]``): the
    per-64-row-tile dw partials are left there and dw is NOT written (``partials_reduce_multi``
    finishes it); ``bias_part`` (same shape): per-tile column sums of g, the last hidden layer's
    bias-gradient partials."""
    if a.is_cuda:
        require().mlp_head(a, w, b0, y, dz, dw, db, loss_acc, g, gT, dw_part, bias_part)
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
    B, D = a.shape
    if dw_part is not None:
        dw_part.copy_((d.view(B // 64, 64, 1) * af.view(B // 64, 64, D)).sum(1))
    if bias_part is not None:
        bias_part.copy_(g.float().view(B // 64, 64, D).sum(1))
