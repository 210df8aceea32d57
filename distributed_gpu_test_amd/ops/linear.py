"""Fused small-batch Linear (+ReLU) for the engine path (``csrc/linear.hip``): kernel injection.

Reference: the model's ``Linear(20,64) -> ReLU -> Linear(64,1)`` (``train.py:29-33``), forward at
``train.py:107``, backward at ``train.py:113``.

Autograd runs a Linear + ReLU as addmm + relu forward and mm + mm + sum + threshold_backward
backward; at the reference's batch of 4 each is a sub-microsecond kernel, and inside a
HIP-graph-replayed step each costs a graph node of a few microseconds.  ``FusedLinear`` does one
launch forward (bias and ReLU folded in) and one launch backward (ReLU mask, dx, dW, db).
``inject_fused_linear(module)`` swaps every ``nn.Linear`` of a module in place — folding an
``nn.ReLU`` that directly follows it in an ``nn.Sequential`` — keeping the same Parameter objects
and state_dict keys, so checkpoints, the engine's flat buffers and optimizers are unaffected.

Every fp32 GPU shape runs a hand-written kernel: small shapes (``SMALL_M`` / ``SMALL_WORK``) the
one-launch dot-product kernels of ``csrc/linear.hip`` (a two-layer chain in one launch each way);
larger ones the exact-fp32 MFMA GEMM of ``csrc/gemm_f32_kernel.h`` (v_mfma_f32_16x16x4_f32,
register-fed, K split inside the workgroup for small grids) -- forward with bias / ReLU in the
epilogue, dgrad and wgrad reading dy, W and x in their stored layouts with the ReLU mask applied
while loading, and the bias gradient as the wgrad's deterministic row sums.  Only
non-fp32 / non-contiguous / CPU inputs run ``F.linear``, and those are counted (``FALLBACKS``).  bf16
models get the MFMA GEMM chain of ``ops/mfma_linear.py`` instead: ``inject_fused_linear``
dispatches on the parameters' dtype.
"""
from __future__ import annotations

import collections
import os
import sys
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..models.synthetic_mlp import SyntheticMLP
from . import _ext
from ..utils.fnapply import fast_apply
from .loss import FREED, keep_graph, release

MODIFIED = ("one of the variables needed for gradient computation has been modified by an inplace operation: "
            "the input or a weight of a fused Linear changed between its forward and this backward")

# > 0 while the engine runs a backward (Engine.backward / the graphed step): only then do the
# in-place kernels add dW / db straight into the parameters' .grad views (the engine's flat
# gradient buckets).  Autograd runs a HIP Function's backward on its device thread, so this is a
# process-wide counter, not a thread-local.  Any other backward -- torch.autograd.grad on the
# parameters, a user's own loss.backward() -- gets dW / db returned to autograd as usual.
_ENGINE_BACKWARD = 0
# the engine's flat gradient buffer is all zeros at the start of this backward (the first micro-step
# after zero_grad): the bf16 MFMA chain then STORES a weight gradient instead of accumulating it --
# the FIRST time that gradient is written in this backward only (a module called twice before one
# backward writes each of its gradients twice: the second write must add)
_GRADS_ZERO = False
_WRITTEN: set = set()
# the engine's per-layer readiness callback (Engine._on_layer_ready) while its backward communicates:
# the fused chains are ONE autograd node for many layers, so autograd's post-accumulate hooks would
# fire for every layer only after the whole chain's backward is queued; the chains call grad_ready()
# right after each layer's dW / db kernels instead, and the bucket reducer launches that layer's
# collective there -- overlapped with the layers below (parallel/reducer.py)
_GRAD_READY = None


def grad_ready(*params) -> None:
    """The gradients of ``params`` (written in place into their .grad views) are complete for this
    backward: their kernels are queued on the current stream."""
    f = _GRAD_READY
    if f is not None:
        for p in params:
            if p is not None:
                f(p)


def grad_ready_on() -> bool:
    return _GRAD_READY is not None


class engine_backward:
    """``with engine_backward(grads_zero, on_ready) as stored``: the engine's backward; ``stored`` is
    the set of ``(data_ptr, numel)`` gradient views STORED (first-written) in it; ``on_ready`` (or None)
    receives each parameter whose in-place gradient a chain has finished (``grad_ready``).  (A class,
    not a generator-based context manager: entered once per eager step, where the host cost is the
    step's cost.)"""

    __slots__ = ("grads_zero", "on_ready", "prev", "prev_written", "prev_ready")

    def __init__(self, grads_zero: bool = False, on_ready=None):
        self.grads_zero = bool(grads_zero)
        self.on_ready = on_ready

    def __enter__(self):
        global _ENGINE_BACKWARD, _GRADS_ZERO, _WRITTEN, _GRAD_READY
        _ENGINE_BACKWARD += 1
        self.prev, _GRADS_ZERO = _GRADS_ZERO, self.grads_zero
        self.prev_written, _WRITTEN = _WRITTEN, set()
        self.prev_ready, _GRAD_READY = _GRAD_READY, self.on_ready
        return _WRITTEN

    def __exit__(self, *exc):
        global _ENGINE_BACKWARD, _GRADS_ZERO, _WRITTEN, _GRAD_READY
        _ENGINE_BACKWARD -= 1
        _GRADS_ZERO = self.prev
        _WRITTEN = self.prev_written
        _GRAD_READY = self.prev_ready
        return False


def _in_place_active() -> bool:
    return _ENGINE_BACKWARD > 0


def _grads_zero() -> bool:
    return _GRADS_ZERO


def _first_write(grad: torch.Tensor) -> bool:
    """True if ``grad`` (a view of the zeroed flat buffer) may be STORED rather than accumulated:
    the buffer was zero when this backward began and nothing has written this view since."""
    if not _GRADS_ZERO:
        return False
    key = (grad.data_ptr(), grad.numel())
    if key in _WRITTEN:
        return False
    _WRITTEN.add(key)
    return True


def _store_both(w_grad: torch.Tensor, b_grad: Optional[torch.Tensor]) -> bool:
    """One accumulate flag for a layer's dW and db (the fp32 kernels take one): True = STORE both
    (their first write of a backward that began on a zeroed -- or deferred, stale -- buffer).  Each
    view is asked once; a mix (a view shared with another layer) zeroes the first-written view and
    accumulates into both."""
    fw = _first_write(w_grad)
    if b_grad is None:
        return fw
    fb = _first_write(b_grad)
    if fw != fb:
        (w_grad if fw else b_grad).zero_()
        return False
    return fw


# Every call that leaves the hand-written kernels for F.linear (hipBLASLt / rocBLAS), by reason:
# the engine reports them (Engine.linear_fallbacks, one stderr warning per reason on rank 0).
FALLBACKS: "collections.Counter[str]" = collections.Counter()
_WARNED: set = set()


def count_fallback(reason: str) -> None:
    FALLBACKS[reason] += 1
    import torch.distributed as dist
    rank0 = not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
    if reason not in _WARNED and rank0:
        _WARNED.add(reason)
        print(f"[dgt] WARNING: Linear falls back to F.linear (vendor BLAS): {reason}", file=sys.stderr, flush=True)

_FUSED_ROWSUM = True     # the wgrad forms db (tests / diagnostics switch to the column-sum pass)
SMALL_M = 256            # rows per call (batch)
SMALL_WORK = 1 << 22     # M * N * K: beyond this the tiled MFMA GEMM (csrc/gemm_f32.hip) wins


def _small(x: torch.Tensor, weight: torch.Tensor) -> bool:
    return x.shape[0] <= SMALL_M and x.shape[0] * weight.shape[0] * weight.shape[1] <= SMALL_WORK


def _skinny(x: torch.Tensor, weight: torch.Tensor) -> bool:
    """A head Linear(K, N <= 4) with whole 64-row blocks: two bandwidth passes over x (``csrc/head.hip``
    skinny_f32), not 64 x 64 MFMA tiles with one useful column.  Checked before ``_small``: the
    small-batch kernels walk K serially per output, 55-75 us for Linear(1024, 1) at M = 256 against
    a few us here (profiles/r6_fp32_head_batch256.txt)."""
    return (weight.shape[0] <= 4 and x.shape[0] % 64 == 0 and x.shape[1] % 32 == 0
            and x.data_ptr() % 16 == 0 and weight.data_ptr() % 16 == 0)


def _chain2(x: torch.Tensor, wb) -> bool:
    """A two-layer chain the one-launch kernels take (csrc/linear.hip linear2_*): both layers within the
    small-batch kernels' range, the hidden activation within the kernel's LDS (M * H <= 4096)."""
    if len(wb) != 4 or not _small(x, wb[0]):
        return False
    M, K, H, O = x.shape[0], x.shape[1], wb[0].shape[0], wb[2].shape[0]
    return M * H <= 4096 and M * H * K + M * O * H <= (1 << 20) and wb[2].shape[1] == H


def _fwd(ops, x, weight, bias, relu: bool) -> torch.Tensor:
    """y = act(x W^T + b): the small-batch kernel, the skinny head kernel or the tiled fp32 MFMA GEMM
    (bias/ReLU epilogue)."""
    y = torch.empty(x.shape[0], weight.shape[0], dtype=torch.float32, device=x.device)
    if _skinny(x, weight):
        ops.skinny_f32_fwd(x, weight, bias, y, relu)
    elif _small(x, weight):
        ops.linear_fwd(x, weight, bias, y, relu)
    else:
        ops.gemm_f32(x, weight, None, bias, y, 0, 0, relu, False)
    return y


def _bwd(ops, dy, x, weight, y, dx, dW, db, accumulate: bool = False, mask_dx=None) -> bool:
    """g = dy * 1[y > 0] (y given: the layer had a ReLU) or dy; dx = g W, dW (+)= g^T x, db (+)= sum_m g.
    Tiled: dgrad A = g [M, N] (k = N contiguous), B = W [N, K] read as [k][n]; wgrad A = g read as
    [k = M][n], B = x [M, K] read as [k][col]; the mask is applied while g is staged, and the wgrad
    sums the staged g per row of A for db (no separate column-sum pass over dy and y).
    ``mask_dx`` (the layer below's ReLU output): the tiled dgrad stores dx * 1[mask_dx > 0], the
    gradient the layer below needs, so that layer reads no mask.  Returns whether it did (the
    small-batch kernel does not)."""
    if _skinny(x, weight) and dW.data_ptr() % 16 == 0 and (mask_dx is None or mask_dx is x):
        ops.skinny_f32_bwd(dy, y, x, weight, mask_dx is not None, dx, dW, db, accumulate)
        return dx is not None and mask_dx is not None
    if _small(x, weight):
        ops.linear_bwd(dy, x, weight, y, dx, dW, db, accumulate)
        return False
    if dx is not None:
        ops.gemm_f32(dy, weight, y, None, dx, 0, 1, False, False, None, mask_dx)
    if _FUSED_ROWSUM:
        # db = the row sums of the wgrad's masked A (g^T), formed while the GEMM stages it
        ops.gemm_f32(dy, x, y, None, dW, 1, 1, False, accumulate, db)
    else:
        ops.gemm_f32(dy, x, y, None, dW, 1, 1, False, accumulate)
        if db is not None:
            ops.colsum_f32(dy, y, db, accumulate)
    return dx is not None and mask_dx is not None


class _FusedLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, relu: bool, grad_in_place: bool = False):
        y = _fwd(_ext.hot(), x, weight, bias, relu)
        ctx.relu = relu
        ctx.has_bias = bias is not None
        # leaf parameters only (no reference cycle through ctx)
        ctx.grad_in_place = grad_in_place and weight.is_leaf and (bias is None or bias.is_leaf)
        ctx.params = (weight, bias) if ctx.grad_in_place else (None, None)
        # the input and the weight as attributes (freed by the direct backward: ops/loss.py
        # release), the output through save_for_backward (an attribute would be a reference cycle)
        ctx.x, ctx.w, ctx.freed, ctx.held = x, weight, False, ("x", "w")
        # (held as attributes, not saved tensors: autograd's in-place check is done here instead)
        ctx.vers = (x._version, weight._version)
        ctx.save_for_backward(y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        if ctx.freed:
            raise RuntimeError(FREED)
        (y,) = ctx.saved_tensors
        x, weight = ctx.x, ctx.w
        if (x._version, weight._version) != ctx.vers:
            raise RuntimeError(MODIFIED)
        if not keep_graph():
            release(ctx)
        dy = dy.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        w_leaf, b_leaf = ctx.params
        if (ctx.grad_in_place and _in_place_active() and ctx.needs_input_grad[1] and w_leaf.requires_grad
                and _grad_view_ok(w_leaf) and (b_leaf is None or (b_leaf.requires_grad and _grad_view_ok(b_leaf)))):
            # write straight into the existing .grad views (the engine's flat bucket; stored on
            # their first write of a from-zero backward, else added): no separate AccumulateGrad
            # add kernel per parameter.  Autograd still runs the leaves'
            # AccumulateGrad nodes with an undefined gradient, which fire the post-accumulate hooks
            # (the engine's bucket reducer) after this kernel is queued
            bg = None if b_leaf is None else b_leaf.grad
            _bwd(_ext.hot(), dy, x, weight, y, dx, w_leaf.grad, bg, not _store_both(w_leaf.grad, bg))
            grad_ready(w_leaf, b_leaf)
            return dx, None, None, None, None
        dw = torch.empty_like(weight)
        db = torch.empty(weight.shape[0], dtype=torch.float32, device=x.device) if ctx.has_bias else None
        _bwd(_ext.hot(), dy, x, weight, y, dx, dw, db)
        return dx, dw, db, None, None


def _grad_view_ok(p, dtype=torch.float32) -> bool:
    g = p.grad
    return (g is not None and g.is_cuda and g.dtype == dtype and g.is_contiguous()
            and g.shape == p.shape and not torch.is_grad_enabled())


def _fusable_param(weight: torch.Tensor, bias=None) -> bool:
    return (weight.dtype == torch.float32 and weight.is_contiguous()
            and (bias is None or (bias.dtype == torch.float32 and bias.is_contiguous())))


def _fusable(x: torch.Tensor, weight: torch.Tensor, bias=None) -> bool:
    return (x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and weight.dtype == torch.float32
            and weight.is_contiguous() and (bias is None or (bias.dtype == torch.float32 and bias.is_contiguous()))
            and _ext.require() is not None)  # a GPU shape we own: a missing extension is an error


def fused_linear(x: torch.Tensor, weight: torch.Tensor, bias=None, relu: bool = False,
                 grad_in_place: bool = False) -> torch.Tensor:
    """``grad_in_place``: inside the engine's backward (``engine_backward``), backward adds dW / db
    into the existing ``.grad`` tensors of leaf parameters instead of returning them to autograd
    (their post-accumulate hooks still fire); any other backward gets them returned as usual."""
    if _fusable(x, weight, bias):
        return _linear_apply(x.contiguous(), weight, bias, relu, grad_in_place)
    if x.is_cuda:
        count_fallback(f"Linear({weight.shape[1]}, {weight.shape[0]}) with {weight.dtype} weights on "
                       f"{tuple(x.shape)} {x.dtype} input (fp32, contiguous parameters only)")
    y = F.linear(x, weight, bias)
    return F.relu(y) if relu else y


class FusedLinear(nn.Linear):
    """``nn.Linear`` (optionally followed by ReLU) on the fused kernels; same parameters and keys."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, relu: bool = False,
                 device=None, dtype=None):
        super().__init__(in_features, out_features, bias=bias, device=device, dtype=dtype)
        self.relu = relu
        self.grad_in_place = False

    @classmethod
    def from_linear(cls, lin: nn.Linear, relu: bool = False, grad_in_place: bool = False) -> "FusedLinear":
        m = cls.__new__(cls)
        nn.Module.__init__(m)
        m.in_features, m.out_features = lin.in_features, lin.out_features
        m.weight = lin.weight          # the same Parameter objects
        m.bias = lin.bias
        m.relu = relu
        m.grad_in_place = grad_in_place
        return m

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shp = x.shape
        y = fused_linear(x.reshape(-1, shp[-1]), self.weight, self.bias, self.relu, self.grad_in_place)
        return y.reshape(*shp[:-1], self.out_features)

    def extra_repr(self) -> str:
        return super().extra_repr() + (", relu=True" if self.relu else "")


class _FusedChainFn(torch.autograd.Function):
    """A chain of fused Linear(+ReLU) layers as ONE autograd node: the forward queues one
    ``linear_fwd`` per layer and the backward one ``linear_bwd`` per layer in reverse, the same
    kernels in the same order as the per-layer path (bit-identical results), but one Function
    apply and one backward node for the whole chain instead of one per layer (the eager engine's
    step is host-bound: profiles/r2_engine_host_profile.txt)."""

    @staticmethod
    def forward(ctx, x, relus, grad_in_place, *wb):
        ops = _ext.hot()
        acts = [x]
        h = x
        ctx.chain2 = _chain2(x, wb)
        if ctx.chain2:
            # the reference model's shape: both layers in ONE launch (csrc/linear.hip linear2_fwd,
            # bitwise the two per-layer launches)
            W1, b1, W2, b2 = wb
            hid = torch.empty(x.shape[0], W1.shape[0], dtype=torch.float32, device=x.device)
            h = torch.empty(x.shape[0], W2.shape[0], dtype=torch.float32, device=x.device)
            ops.linear2_fwd(x, W1, b1, W2, b2, hid, h, relus[0], relus[1])
            acts += [hid, h]
        for i, relu in enumerate(relus if not ctx.chain2 else ()):
            y = _fwd(ops, h, wb[2 * i], wb[2 * i + 1], relu)
            acts.append(y)
            h = y
        ctx.relus = relus
        ctx.has_bias = tuple(b is not None for b in wb[1::2])
        ctx.grad_in_place = grad_in_place and all(p is None or p.is_leaf for p in wb)
        ctx.params = wb if ctx.grad_in_place else ()
        # the input, the hidden activations and the weights as attributes (none of them an output:
        # no reference cycle; freed by the direct backward, ops/loss.py release), the chain's output
        # through save_for_backward
        ctx.acts, ctx.ws, ctx.freed, ctx.held = acts[:-1], wb[0::2], False, ("acts", "ws")
        # (the hidden activations are the chain's own; the input and the weights are the caller's)
        ctx.vers = (x._version, *[w._version for w in wb[0::2]])
        ctx.save_for_backward(h)
        return h

    @staticmethod
    def backward(ctx, dy):
        ops = _ext.hot()
        if ctx.freed:
            raise RuntimeError(FREED)
        L = len(ctx.relus)
        acts, ws = list(ctx.acts) + list(ctx.saved_tensors), ctx.ws
        if (acts[0]._version, *[w._version for w in ws]) != ctx.vers:
            raise RuntimeError(MODIFIED)
        if not keep_graph():
            release(ctx)
        active = ctx.grad_in_place and _in_place_active()
        if ctx.chain2 and active and all(ctx.needs_input_grad[3:3 + 2 * L:2]):
            # both layers' gradients into their .grad views in ONE launch (csrc/linear.hip linear2_bwd)
            W1, W2 = ctx.params[0], ctx.params[2]
            B1, B2 = ctx.params[1], ctx.params[3]
            if (all(_grad_view_ok(p) for p in (W1, W2)) and all(b is None or (b.requires_grad and _grad_view_ok(b))
                                                                for b in (B1, B2))):
                acc2 = not _store_both(W2.grad, None if B2 is None else B2.grad)
                acc1 = not _store_both(W1.grad, None if B1 is None else B1.grad)
                dx = torch.empty_like(acts[0]) if ctx.needs_input_grad[0] else None
                ops.linear2_bwd(dy.contiguous(), acts[0], ws[0], acts[1], ws[1], acts[2] if ctx.relus[1] else None, dx,
                                W1.grad, None if B1 is None else B1.grad, W2.grad, None if B2 is None else B2.grad,
                                ctx.relus[0], acc1, acc2)
                grad_ready(W2, B2, W1, B1)
                return (dx, None, None, *([None] * (2 * L)))
        grads = [None] * (2 * L)
        dy = dy.contiguous()
        masked = False  # dy already carries this layer's ReLU mask (stored so by the dgrad above)
        for i in reversed(range(L)):
            dx = torch.empty_like(acts[i]) if (i > 0 or ctx.needs_input_grad[0]) else None
            y = acts[i + 1] if ctx.relus[i] and not masked else None
            # the layer below's ReLU mask goes into this dgrad's store (i > 0: dx feeds layer i - 1)
            mask_dx = acts[i] if (i > 0 and ctx.relus[i - 1]) else None
            # per layer: a parameter frozen after injection (requires_grad False) gets nothing, and
            # only a layer whose trained tensors all have live .grad views accumulates in place
            w_need, b_need = ctx.needs_input_grad[3 + 2 * i], ctx.has_bias[i] and ctx.needs_input_grad[4 + 2 * i]
            w_leaf = ctx.params[2 * i] if active else None
            b_leaf = ctx.params[2 * i + 1] if active else None
            in_place = (active and w_need and _grad_view_ok(w_leaf)
                        and (not ctx.has_bias[i] or (b_need and _grad_view_ok(b_leaf))))
            if in_place:
                bg = None if b_leaf is None else b_leaf.grad
                masked = _bwd(ops, dy, acts[i], ws[i], y, dx, w_leaf.grad, bg, not _store_both(w_leaf.grad, bg),
                              mask_dx)
                grad_ready(w_leaf, b_leaf)  # this layer's bucket may go out while the layers below run
            else:
                dw = torch.empty_like(ws[i])
                db = torch.empty(ws[i].shape[0], dtype=torch.float32, device=dy.device) if ctx.has_bias[i] else None
                masked = _bwd(ops, dy, acts[i], ws[i], y, dx, dw, db, mask_dx=mask_dx)
                grads[2 * i] = dw if w_need else None
                grads[2 * i + 1] = db if b_need else None
            dy = dx
        return (dy, None, None, *grads)


class FusedChain(nn.Sequential):
    """An ``nn.Sequential`` whose children are all ``FusedLinear`` (folded ReLUs left as
    ``nn.Identity``): a 2-D fp32 GPU input every layer can take runs as one ``_FusedChainFn``;
    anything else runs layer by layer.  Same children, keys and parameters as the Sequential."""

    def _chain(self):
        layers = [m for m in self if not isinstance(m, nn.Identity)]
        return layers if layers and all(isinstance(m, FusedLinear) for m in layers) else None

    def forward(self, x):
        layers = self.__dict__.get("_dgt_layers")
        if layers is None:
            layers = self._chain() or []
            self.__dict__["_dgt_layers"] = layers
        if len(layers) > 1 and x.dim() == 2 and x.is_cuda and x.dtype == torch.float32:
            # (the parameters straight from each layer's _parameters: nn.Module.__getattr__ is a
            # measurable part of a host-bound eager step)
            wb = []
            ok = True
            for m in layers:
                w, b = m._parameters["weight"], m._parameters["bias"]
                if not _fusable_param(w, b):
                    ok = False
                    break
                wb.append(w)
                wb.append(b)
            if ok and _ext.require() is not None:
                relus = self.__dict__.get("_dgt_relus")
                if relus is None:
                    relus = self.__dict__["_dgt_relus"] = tuple(m.relu for m in layers)
                return _chain_apply(x.contiguous(), relus, layers[0].grad_in_place, *wb)
        return super().forward(x)


class FusedSyntheticMLP(SyntheticMLP):
    """``SyntheticMLP`` (``layers`` each followed by ReLU, then ``head``; its ReLU is a
    ``torch.relu`` call in ``forward``, not a module, so the Sequential folding above cannot see it)
    as one ``_FusedChainFn``: the ReLUs go into the GEMM epilogues and the dgrads' staging masks,
    and the whole model is one autograd node.  Installed by swapping the instance's class (same
    children, keys and parameters); inputs the chain cannot take run layer
    by layer (the layers are ``FusedLinear(relu=True)``, so no second ReLU is applied)."""

    def forward(self, x):
        layers = list(self.layers) + [self.head]
        if x.dim() == 2 and all(isinstance(m, FusedLinear) and _fusable(x, m.weight, m.bias) for m in layers):
            wb = []
            for m in layers:
                wb.append(m.weight)
                wb.append(m.bias)
            return _chain_apply(x.contiguous(), tuple(m.relu for m in layers), layers[0].grad_in_place, *wb)
        for m in self.layers:
            x = m(x)
        return self.head(x)


def _fuse_synthetic_mlp(module: nn.Module, grad_in_place: bool) -> int:
    for i, lin in enumerate(module.layers):
        module.layers[i] = FusedLinear.from_linear(lin, relu=True, grad_in_place=grad_in_place)
    module.head = FusedLinear.from_linear(module.head, grad_in_place=grad_in_place)
    module.__class__ = FusedSyntheticMLP
    return len(module.layers) + 1


def inject_fused_linear(module: nn.Module, grad_in_place: bool = False) -> int:
    """Replace nn.Linear (+ a directly following nn.ReLU inside an nn.Sequential) in place,
    recursively; ``module`` itself may be the Sequential.  A plain ``nn.Sequential`` left holding
    only fused layers becomes a ``FusedChain`` (its class is swapped in place, so the object, its
    children and keys stay the same).  Returns the number of Linear layers replaced.
    ``grad_in_place``: see ``fused_linear`` (the engine sets it: its .grad tensors are persistent
    views into the flat gradient bucket).  A bf16 module goes to the MFMA chain injection
    (``ops/mfma_linear.py``)."""
    p = next(module.parameters(), None)
    if p is not None and p.dtype == torch.bfloat16:
        from .mfma_linear import inject_mfma_linear
        return inject_mfma_linear(module, grad_in_place)
    if type(module) is SyntheticMLP and all(type(m) is nn.Linear for m in module.layers) \
            and type(module.head) is nn.Linear:
        return _fuse_synthetic_mlp(module, grad_in_place)
    n = 0
    if isinstance(module, nn.Sequential):
        kids = list(module.children())
        for i, k in enumerate(kids):
            if type(k) is nn.Linear:
                fold = i + 1 < len(kids) and type(kids[i + 1]) is nn.ReLU
                module[i] = FusedLinear.from_linear(k, relu=fold, grad_in_place=grad_in_place)
                if fold:
                    module[i + 1] = nn.Identity()
                n += 1
            elif not isinstance(k, FusedLinear):
                n += inject_fused_linear(k, grad_in_place)
        if type(module) is nn.Sequential and FusedChain._chain(module):
            module.__class__ = FusedChain
        return n
    for name, child in list(module.named_children()):
        if type(child) is nn.Linear:
            setattr(module, name, FusedLinear.from_linear(child, grad_in_place=grad_in_place))
            n += 1
        elif not isinstance(child, FusedLinear):
            n += inject_fused_linear(child, grad_in_place)
    return n


_linear_apply = fast_apply(_FusedLinearFn)
_chain_apply = fast_apply(_FusedChainFn)
