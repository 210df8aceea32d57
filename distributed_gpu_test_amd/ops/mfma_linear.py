"""bf16 Linear(+ReLU) chains on the hand-written MFMA GEMMs, for the engine's bf16 path.

Reference: the model's ``Linear -> ReLU -> Linear`` (``train.py:29-33``), forward at
``train.py:107`` and backward at ``train.py:113``, scaled to the bench MLP (BASELINE config #2).

Left to autograd, a bf16 ``nn.Linear`` runs ``F.linear`` = hipBLASLt (``Cijk_*`` kernels) plus
separate bias, ReLU and ReLU-backward elementwise passes.  A chain of layers here is ONE autograd
node whose kernels are this framework's (``csrc/gemm.hip``, ``csrc/head.hip``):

    forward   y_i = relu(x_i W_i^T + b_i)          gemm_nt, bias + ReLU epilogue, plus y_i^T (the next
                                                   layer's wgrad operand) from the same epilogue
    head      z = y_L w^T + b  (N <= 4 outputs)    skinny_fwd_bf16
    backward  g_L = (dz w) * 1[y_L > 0], g_L^T     skinny_bwd_bf16 (+ the head's dw, db)
              dW_i = g_i^T x_i  -> the .grad view   gemm_nt (stores into the engine's flat bf16
                                                   gradient bucket; accumulates after the first
                                                   micro-step of an accumulation window)
              db_i = column sums of g_i             per-row-tile partials from the kernel that forms
                                                   g_i (skinny_bwd / the dgrad epilogue's colsum),
                                                   all layers reduced by ONE partials_reduce_multi
                                                   (fixed order, bf16 out); rowsum_bf16 of g_i^T when
                                                   no partials exist (no ReLU below the layer)
              g_{i-1} = (g_i W_i) * 1[x_i > 0], g^T  gemm_nt reading W_i[out, in] as a [K, N] operand
                                                   (transposed LDS reads), mask + C^T epilogue

Inside the engine's backward (``ops.linear.engine_backward``) the gradients land straight in the
parameters' ``.grad`` views; any other backward gets them returned to autograd.  Structures
recognised: an ``nn.Sequential`` of ``Linear[, ReLU]`` ... ending in a ``Linear`` (MFMA-sized or a
skinny head), and ``SyntheticMLP`` (``layers`` + ReLU + ``head``).  MFMA-sized means in and out
features multiples of 128; at run time the batch must be a multiple of 128 too.  Anything else
runs the module's own forward (``F.linear``) and is counted in ``ops.linear.FALLBACKS``.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from ..models.synthetic_mlp import SyntheticMLP
from .gemm import gemm_nt, partials_reduce_multi, rowsum_bf16, skinny_bwd_bf16, skinny_fwd_bf16, transpose_bf16
from ..utils.fnapply import fast_apply
from .linear import _first_write, _grad_view_ok, _in_place_active, count_fallback, grad_ready, grad_ready_on

MAX_HEAD = 4
BF16 = torch.bfloat16


def _mfma_sized(lin: nn.Linear) -> bool:
    return lin.in_features % 128 == 0 and lin.out_features % 128 == 0


def _head_sized(lin: nn.Linear) -> bool:
    return lin.out_features <= MAX_HEAD and lin.in_features % 128 == 0


def chain_layout(linears: Sequence[nn.Linear], relus: Sequence[bool]) -> Optional[bool]:
    """None if the chain cannot run on the kernels, else whether its last Linear is a skinny head."""
    if not linears or len(linears) != len(relus):
        return None
    head = not _mfma_sized(linears[-1])
    body = linears[:-1] if head else linears
    if not body or not all(_mfma_sized(l) for l in body):
        return None
    if head and (relus[-1] or not _head_sized(linears[-1])):
        return None
    for a, b in zip(linears, linears[1:]):
        if a.out_features != b.in_features:
            return None
    return head


_ZERO_BIAS: dict = {}


def _zero_bias(n: int, device) -> torch.Tensor:
    key = (n, str(device))
    z = _ZERO_BIAS.get(key)
    if z is None:
        z = _ZERO_BIAS[key] = torch.zeros(n, dtype=BF16, device=device)
    return z


def _runtime_reason(x: torch.Tensor, params: Sequence[Optional[torch.Tensor]]) -> Optional[str]:
    if not x.is_cuda or x.dtype != BF16 or x.dim() != 2:
        return f"input {tuple(x.shape)} {x.dtype} on {x.device.type} is not a 2-D bf16 GPU tensor"
    if x.shape[0] % 128:
        return f"batch {x.shape[0]} is not a multiple of 128 (the MFMA GEMM's tile)"
    for p in params:
        if p is not None and (p.dtype != BF16 or not p.is_contiguous() or p.data_ptr() % 16):
            return "a parameter is not a contiguous, 16-byte aligned bf16 tensor"
    return None


class _MfmaChainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, relus, head, grad_in_place, *wb):
        L = len(relus) - (1 if head else 0)  # MFMA layers; the head (if any) is the last pair of wb
        need = ctx.needs_input_grad
        M, dev = x.shape[0], x.device
        xs: List[torch.Tensor] = [x]
        xTs: List[Optional[torch.Tensor]] = [None] * L
        if need[4]:  # layer 0's wgrad reads x^T
            xTs[0] = torch.empty(x.shape[1], M, dtype=BF16, device=dev)
            transpose_bf16(x, xTs[0])
        h = x
        for i in range(L):
            w, b = wb[2 * i], wb[2 * i + 1]
            y = torch.empty(M, w.shape[0], dtype=BF16, device=dev)
            yT = None
            if i + 1 < L and need[4 + 2 * (i + 1)]:
                yT = xTs[i + 1] = torch.empty(w.shape[0], M, dtype=BF16, device=dev)
            # a bf16 bias is read as it is; a bias-less Linear reads a zero bias (the GEMM's epilogue
            # set has every ReLU / C^T form only with the bias add: x + 0 is x)
            gemm_nt(h, w, C=y, CT=yT, bias=b if b is not None else _zero_bias(w.shape[0], dev), relu=relus[i])
            xs.append(y)
            h = y
        out = h
        if head:
            wh, bh = wb[2 * L], wb[2 * L + 1]
            out = torch.empty(M, wh.shape[0], dtype=BF16, device=dev)
            skinny_fwd_bf16(h, wh, bh, out)
        ctx.relus, ctx.head, ctx.L = tuple(relus), bool(head), L
        ctx.has_bias = tuple(b is not None for b in wb[1::2])
        ctx.grad_in_place = grad_in_place and all(p is None or p.is_leaf for p in wb)
        ctx.params = wb if ctx.grad_in_place else ()
        ctx.save_for_backward(*xs, *xTs, *wb[0::2])
        return out

    @staticmethod
    def backward(ctx, dout):
        L, head, relus = ctx.L, ctx.head, ctx.relus
        saved = ctx.saved_tensors
        xs, xTs, ws = saved[:L + 1], saved[L + 1:2 * L + 1], saved[2 * L + 1:]
        need = ctx.needs_input_grad
        active = ctx.grad_in_place and _in_place_active()
        M, dev = xs[0].shape[0], xs[0].device
        n_pairs = L + (1 if head else 0)
        grads: List[Optional[torch.Tensor]] = [None] * (2 * n_pairs)
        dout = dout.to(BF16).contiguous()

        def leaf(j):
            return ctx.params[j] if active else None

        def wants_bias(i):  # layer i's bias gradient is needed
            return ctx.has_bias[i] and need[4 + 2 * i + 1]

        bpart = None  # column-sum partials of the current g (fp32 [row tiles, features]), if formed
        segs = []     # (partials, bias-gradient target, accumulate): reduced together at the end
        # the engine's backward communicates (ops.linear.grad_ready): each layer's partials are reduced
        # right after its wgrad and the layer is reported complete there, so its bucket's collective
        # overlaps the layers below; else every layer's partials go into one launch at the end
        notify = active and grad_ready_on()
        if head:
            wh = ws[L]
            kh = wh.shape[1]
            g = torch.empty(M, kh, dtype=BF16, device=dev)
            gT = torch.empty(kh, M, dtype=BF16, device=dev)
            jw, jb = 2 * L, 2 * L + 1
            pw, pb = leaf(jw), (leaf(jb) if ctx.has_bias[L] else None)
            mask_h = relus[L - 1] if L > 0 else False
            hb = torch.empty(M // 64, kh, dtype=torch.float32, device=dev) if L > 0 and wants_bias(L - 1) else None
            direct = (need[4 + jw] and pw is not None and _grad_view_ok(pw, BF16)
                      and (not ctx.has_bias[L] or (need[4 + jb] and pb is not None and _grad_view_ok(pb, BF16))))
            firsts = {}  # _first_write decisions already taken (each view is asked once per backward)
            if direct:
                store_w = firsts[jw] = _first_write(pw.grad)
                store_b = _first_write(pb.grad) if pb is not None else store_w
                if pb is not None:
                    firsts[jb] = store_b
                direct = store_w == store_b  # (else: the per-tensor store / add path below)
            if direct:
                # straight into the bucket's bf16 views, stored on their first write of this backward
                db = pb.grad if pb is not None else torch.zeros(wh.shape[0], dtype=BF16, device=dev)
                # dW's row-tile partials join the one reduction launch at the end (bias gradients)
                hw = (torch.empty(M // 64, wh.numel(), dtype=torch.float32, device=dev)
                      if pw.grad.data_ptr() % 8 == 0 else None)
                skinny_bwd_bf16(dout, xs[L], wh, mask_h, g, gT, pw.grad, db, accumulate=not store_w, bias_part=hb,
                                dw_part=hw)
                if hw is not None:
                    segs.append((hw, pw.grad.view(-1), not store_w))
                if notify:
                    if segs:
                        partials_reduce_multi(segs)
                        segs = []
                    grad_ready(pw, pb)
            else:
                dw = torch.zeros(wh.shape, dtype=torch.float32, device=dev)
                db = torch.zeros(wh.shape[0], dtype=torch.float32, device=dev)
                skinny_bwd_bf16(dout, xs[L], wh, mask_h, g, gT, dw, db, bias_part=hb)
                for j, val in ((jw, dw), (jb, db)):
                    if j == jb and not ctx.has_bias[L]:
                        continue
                    if not need[4 + j]:
                        continue
                    p = leaf(j)
                    if p is not None and _grad_view_ok(p, BF16):
                        # tiny: [N <= 4, K] and [N].  A first write of this backward STORES: the
                        # view may be a deferred (stale) buffer the engine has not zeroed
                        first = firsts[j] if j in firsts else _first_write(p.grad)
                        if first:
                            p.grad.copy_(val)
                        else:
                            p.grad.add_(val)
                    else:
                        grads[j] = val.to(BF16)
            bpart = hb
        else:
            y = xs[L]
            g = (dout * (y > 0)).contiguous() if relus[L - 1] else dout
            gT = torch.empty(g.shape[1], M, dtype=BF16, device=dev)
            transpose_bf16(g, gT)
        dx = None
        for i in reversed(range(L)):
            w = ws[i]
            jw, jb = 2 * i, 2 * i + 1
            done = []  # parameters of this layer written in place (reported to the engine below)
            if need[4 + jw]:
                p = leaf(jw)
                if p is not None and _grad_view_ok(p, BF16):
                    gemm_nt(gT, xTs[i], C=p.grad, accumulate=not _first_write(p.grad))
                    done.append(p)
                else:
                    grads[jw] = torch.empty_like(w)
                    gemm_nt(gT, xTs[i], C=grads[jw])
            if wants_bias(i):
                p = leaf(jb)
                if p is not None and _grad_view_ok(p, BF16) and (bpart is None or p.grad.data_ptr() % 8 == 0):
                    tgt, acc = p.grad, not _first_write(p.grad)
                    done.append(p)
                else:
                    tgt = grads[jb] = torch.empty(w.shape[0], dtype=BF16, device=dev)
                    acc = False
                if bpart is not None:
                    segs.append((bpart, tgt, acc))
                else:
                    rowsum_bf16(gT, tgt, accumulate=acc)
            if notify:
                if segs:
                    partials_reduce_multi(segs)
                    segs = []
                grad_ready(*done)
            if i > 0:
                k = w.shape[1]
                g_prev = torch.empty(M, k, dtype=BF16, device=dev)
                gT_prev = torch.empty(k, M, dtype=BF16, device=dev)
                bpart = None
                if relus[i - 1] and wants_bias(i - 1):  # the epilogue's colsum needs the ReLU mask
                    bpart = torch.empty(M // 128, k, dtype=torch.float32, device=dev)
                gemm_nt(g, w, C=g_prev, CT=gT_prev, mask=xs[i] if relus[i - 1] else None, b_kn=True,
                        colsum=bpart)
                g, gT = g_prev, gT_prev
            elif need[0]:
                dx = torch.empty_like(xs[0])
                gemm_nt(g, w, C=dx, b_kn=True)
        for s0 in range(0, len(segs), 8):
            partials_reduce_multi(segs[s0:s0 + 8])
        return (dx, None, None, None, *grads)


def run_chain(x: torch.Tensor, linears: Sequence[nn.Linear], relus: Sequence[bool], head: bool,
              grad_in_place: bool) -> Optional[torch.Tensor]:
    """The chain on the kernels, or None (after counting the reason) if this call cannot run there."""
    wb = []
    for l in linears:
        wb.append(l.weight)
        wb.append(l.bias)
    why = _runtime_reason(x, wb)
    if why is None and x.requires_grad and linears[0].in_features % 128:
        why = "the input needs a gradient and its features are not a multiple of 128"
    if why is not None:
        count_fallback(f"bf16 MFMA chain: {why}")
        return None
    return _mfma_chain_apply(x.contiguous(), tuple(relus), head, grad_in_place, *wb)


class MfmaSequential(nn.Sequential):
    """An ``nn.Sequential`` of ``Linear[, ReLU]`` ... ``Linear`` run as one MFMA chain (same children,
    keys and parameters; the class is swapped in place by ``inject_mfma_linear``)."""

    def _spec(self):
        spec = self.__dict__.get("_dgt_spec")
        if spec is None:
            kids = list(self.children())
            linears, relus, ok = [], [], True
            for k in kids:
                if type(k) is nn.Linear:
                    linears.append(k)
                    relus.append(False)
                elif type(k) is nn.ReLU and linears and not relus[-1]:
                    relus[-1] = True
                else:
                    ok = False
            head = chain_layout(linears, relus) if ok else None
            spec = (linears, relus, head)
            self.__dict__["_dgt_spec"] = spec
        return spec

    def forward(self, x):
        linears, relus, head = self._spec()
        if head is not None and x.dim() == 2:
            out = run_chain(x, linears, relus, head, self.__dict__.get("_dgt_in_place", False))
            if out is not None:
                return out
        return super().forward(x)


class MfmaSyntheticMLP(SyntheticMLP):
    """``SyntheticMLP`` (``layers`` each followed by ReLU, then ``head``) as one MFMA chain."""

    def forward(self, x):
        linears = list(self.layers) + [self.head]
        relus = [True] * len(self.layers) + [False]
        head = chain_layout(linears, relus)
        if head is not None and x.dim() == 2:
            out = run_chain(x, linears, relus, head, self.__dict__.get("_dgt_in_place", False))
            if out is not None:
                return out
        return super().forward(x)


def inject_mfma_linear(module: nn.Module, grad_in_place: bool = False) -> int:
    """Swap every recognised bf16 chain inside ``module`` (or ``module`` itself) for its MFMA form,
    in place: same objects, children, parameters and state_dict keys.  Returns the number of Linear
    layers that run on the kernels; a chain that does not fit is left alone and counted."""
    if type(module) is SyntheticMLP:
        linears = list(module.layers) + [module.head]
        if chain_layout(linears, [True] * len(module.layers) + [False]) is None:
            count_fallback(f"bf16 SyntheticMLP(width={module.width}) is not MFMA-sized (multiples of 128)")
            return 0
        module.__class__ = MfmaSyntheticMLP
        module.__dict__["_dgt_in_place"] = grad_in_place
        return len(linears)
    if type(module) is nn.Sequential:
        module.__class__ = MfmaSequential
        linears, relus, head = module._spec()
        if head is not None:
            module.__dict__["_dgt_in_place"] = grad_in_place
            return len(linears)
        module.__class__ = nn.Sequential  # not a chain: look inside instead
        module.__dict__.pop("_dgt_spec", None)
    n = 0
    for child in module.children():
        n += inject_mfma_linear(child, grad_in_place)
    if n == 0 and type(module) is nn.Linear:
        count_fallback(f"bf16 Linear({module.in_features}, {module.out_features}) outside a recognised chain")
    return n


_mfma_chain_apply = fast_apply(_MfmaChainFn)
