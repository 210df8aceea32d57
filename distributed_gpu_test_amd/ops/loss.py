"""Fused BCE-with-logits loss (``csrc/loss.hip``) for the engine path.

Reference: ``nn.BCEWithLogitsLoss()`` created at ``train.py:96`` and applied at ``train.py:112``.

One HIP kernel computes the mean loss AND d loss / d logits (saved for backward); backward is one
multiply by the incoming gradient.  torch's loss runs ~11 small kernels per step, and inside a
HIP-graph-replayed step every node costs a few microseconds whatever it computes.  On CPU tensors
(or without the extension) it is ``F.binary_cross_entropy_with_logits`` itself.

Backward seeded with :func:`unit_seed` (the engine's persistent 1, never written) launches nothing:
the gradient IS the saved d loss / d logits -- for bf16 logits the copy the kernel rounded once,
bit for bit what ``dz * 1`` cast to bf16 gives.  Any other seed is one multiply.

d loss / d logits is kept on the node as a plain attribute (it is an intermediate, not an output:
no reference cycle) rather than through ``save_for_backward``, so the engine's direct backward
(``engine._direct_backward``, which calls the node without the autograd engine) can free it the way
autograd frees saved tensors; a backward that does not retain the graph frees it itself.  A second
backward through a freed node raises autograd's own error.  With ``retain_graph`` the unit-seed
path hands out a copy, so a consumer that edits its incoming gradient in place cannot alter the
value a later backward reads.
"""
from __future__ import annotations

import threading
from typing import Optional

import torch
import torch.nn.functional as F
import torch.nn.modules.module as _mod

from . import _ext
from ..utils.fnapply import fast_apply

_UNIT: dict = {}


def unit_seed(device: torch.device) -> torch.Tensor:
    """A persistent fp32 scalar 1 on ``device``; callers must never write it (the BCE backward
    recognises it and skips its multiply)."""
    t = _UNIT.get(device)
    if t is None:
        t = _UNIT[device] = torch.ones((), dtype=torch.float32, device=device)
    return t


FREED = ("Trying to backward through the graph a second time (or directly access saved tensors after they "
         "have already been freed). Saved intermediate values of the graph are freed when you call .backward() "
         "or autograd.grad(). Specify retain_graph=True if you need to backward through the graph a second time "
         "or if you need to access saved tensors after calling backward.")


_DIRECT = threading.local()


def keep_graph() -> bool:
    """Whether the running backward retains the graph: False inside :func:`direct_backward` (the
    engine calling the nodes itself, never retaining), else autograd's answer (True outside any
    backward)."""
    if getattr(_DIRECT, "on", False):
        return False
    if _KEEP is None:  # a torch without the query: assume retained (frees nothing early; compat.py)
        return True
    return _KEEP()


_KEEP = getattr(getattr(torch._C, "_autograd", None), "_get_current_graph_task_keep_graph", None)


class direct_backward:
    """Marks the engine's own calls of the nodes' backward (``engine._direct_backward``): a
    backward that does not retain the graph."""

    __slots__ = ()

    def __enter__(self):
        _DIRECT.on = True

    def __exit__(self, *exc):
        _DIRECT.on = False
        return False


def release(node) -> None:
    """Free what the framework's fused loss / Linear nodes hold for backward (the direct backward's
    counterpart of autograd's release of saved tensors).  Each node lists its attributes in ``held``."""
    held = getattr(node, "held", None)
    if held is not None:
        for attr in held:
            setattr(node, attr, None)
        node.freed = True


_GOUT_ALIAS: dict = {}  # data_ptr of a graphed module's static output -> weakref to its GraphedModule


def register_gout_alias(out: torch.Tensor, runner) -> None:
    """runtime/graph_module.py: logits at ``out``'s address may take their d loss / d logits buffer
    from ``runner.claim_gout`` (the backward graph's static input)."""
    import weakref
    _GOUT_ALIAS[out.data_ptr()] = weakref.ref(runner)


def _gout_buffer(z: torch.Tensor, dtype: torch.dtype) -> Optional[torch.Tensor]:
    ref = _GOUT_ALIAS.get(z.data_ptr()) if _GOUT_ALIAS else None
    runner = ref() if ref is not None else None
    return None if runner is None else runner.claim_gout(z, dtype)


def _is_unit(g: torch.Tensor) -> bool:
    t = _UNIT.get(g.device)
    return t is not None and g.dim() == 0 and g.dtype == torch.float32 and g.data_ptr() == t.data_ptr()


class _FusedBCEWithLogits(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z: torch.Tensor, y: torch.Tensor, sum_into=None) -> torch.Tensor:
        # the kernel reads z and y as flat contiguous arrays of the same length (any shapes); the
        # common case -- contiguous logits, fp32 targets -- passes both as they are (host-bound step)
        zc = z if z.is_contiguous() else z.contiguous()
        yc = y if (y.dtype == torch.float32 and y.is_contiguous()) else y.to(torch.float32).contiguous()
        dev = z.device
        loss = torch.empty((), dtype=torch.float32, device=dev)
        # the gradient a graphed module's backward replays from: written in place when z is that
        # module's fresh output (fp32: dz itself, bf16: the once-rounded copy)
        gbuf = _gout_buffer(zc, z.dtype) if _GOUT_ALIAS else None
        if z.dtype == torch.bfloat16:
            dz = torch.empty(zc.shape, dtype=torch.float32, device=dev)
            lp = gbuf if gbuf is not None else torch.empty(zc.shape, dtype=torch.bfloat16, device=dev)
        else:
            dz = gbuf if gbuf is not None else torch.empty(zc.shape, dtype=torch.float32, device=dev)
            lp = None
        _ext.hot().bce_logits(zc, yc, loss, dz, lp, sum_into)
        ctx.dz, ctx.lp, ctx.freed, ctx.held = dz, lp, False, ("dz", "lp")
        ctx.shape, ctx.dtype = z.shape, z.dtype
        ctx.claimed = gbuf is not None
        return loss

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        if ctx.freed:
            raise RuntimeError(FREED)
        dz, lp = ctx.dz, ctx.lp
        keep = keep_graph()
        if not keep:
            release(ctx)
        elif ctx.claimed:
            # the claimed buffer is the graphed backward's static input: the replay this backward
            # feeds copies its (possibly scaled) gradient there, over what a later backward through
            # this retained graph must read -- keep a private copy for that one
            if lp is not None:
                ctx.lp = lp = lp.clone()
            else:
                ctx.dz = dz = dz.clone()
            ctx.claimed = False
        if _is_unit(g):
            out = (lp if lp is not None else dz).view(ctx.shape)
            return (out.clone() if keep else out), None, None
        # scaled and cast to the logits' dtype in one pass (the fp32 product, rounded once)
        gz = torch.empty(ctx.shape, dtype=ctx.dtype, device=dz.device)
        torch.mul(dz.view(ctx.shape), g, out=gz)
        return gz, None, None


_bce_apply = fast_apply(_FusedBCEWithLogits)


def bce_with_logits(z: torch.Tensor, y: torch.Tensor, sum_into: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Mean BCE-with-logits; the fused HIP kernel on GPU fp32 / bf16 logits.  ``sum_into`` (one fp64
    element on the logits' device): the loss is also added to it -- a training loop's running loss
    log (the reference's per-step ``loss.item()`` sum, train.py:115) as ``sum_into += loss``, inside
    the loss kernel instead of a launch of its own."""
    if sum_into is not None and (sum_into.dtype != torch.float64 or sum_into.numel() != 1
                                 or sum_into.device != z.device):
        raise ValueError("bce_with_logits: sum_into must be one fp64 element on the logits' device")
    if (z.is_cuda and z.dtype in (torch.float32, torch.bfloat16) and z.numel() == y.numel() and z.numel() > 0
            and _ext.require() is not None):  # on the GPU a missing extension is an error, not a fallback
        return _bce_apply(z, y, sum_into)
    loss = F.binary_cross_entropy_with_logits(z, y.to(z.dtype))
    if sum_into is not None:
        sum_into.add_(loss.detach())
    return loss


class BCEWithLogitsLoss(torch.nn.Module):
    """Drop-in for ``nn.BCEWithLogitsLoss()`` (mean reduction, no weights); ``sum_into``: see
    :func:`bce_with_logits`."""

    def __init__(self, sum_into: Optional[torch.Tensor] = None):
        super().__init__()
        self.sum_into = sum_into

    def forward(self, z: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        return bce_with_logits(z, y, self.sum_into)

    def __call__(self, z: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        # straight to forward when no hook could see the call (nn.Module's dispatch is ~1.5 us of a
        # host-bound engine step); with any module or global hook, nn.Module's own call path
        if (self._forward_hooks or self._forward_pre_hooks or self._backward_hooks or self._backward_pre_hooks
                or _mod._global_forward_hooks or _mod._global_forward_pre_hooks or _mod._global_backward_hooks
                or _mod._global_backward_pre_hooks):
            return super().__call__(z, y)
        return bce_with_logits(z, y, self.sum_into)
