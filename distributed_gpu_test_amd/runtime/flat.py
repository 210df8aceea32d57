"""Flat, bucket-aligned parameter and gradient storage.

Reference: parameters moved/broadcast by ``deepspeed.initialize`` (``train.py:87-93``), grads reduced at ``train.py:113``.

DeepSpeed (stage 0) keeps per-tensor ``.grad``s and, at the accumulation boundary, flattens them
into a bucket, all-reduces, scales and unflattens back.  Here every parameter and
gradient is a VIEW into one contiguous buffer from the start, so:

* a bucket is a contiguous slice of the gradient buffer -> RCCL reduces it in place, no
  flatten/unflatten kernels;
* the optimizer is ONE fused launch over the flat buffer (``ops.adam_flat_``);
* for ZeRO-1/2 each bucket is padded to a multiple of ``world_size * 16`` elements so every
  rank's shard of every bucket is contiguous and 64-byte aligned; the concatenation of a rank's
  shards is its contiguous optimizer partition.

Buckets are formed in REVERSE parameter order (backward produces gradients last-layer-first) and
laid out forward, so the first bucket whose gradients are complete is the tail of the buffer.
``units`` (the engine passes one per module: a layer's weight and bias) are never split across
buckets: a layer larger than the bucket size gets a bucket of its own, with its bias in it, so the
layer's collective starts as soon as that layer's backward has written both (``ops/linear.py``
grad_ready) -- not one extra bias-sized collective per layer.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence, Tuple

import torch

ALIGN = 16  # elements: 64 B for fp32, every view 16-byte aligned for float4 / bf16x8 access


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass
class Bucket:
    index: int
    start: int          # element offset in the flat buffer
    numel: int          # padded length
    params: List[int]   # parameter indices (forward order)

    def shard(self, rank: int, world: int) -> Tuple[int, int]:
        n = self.numel // world
        return self.start + rank * n, n


class FlatLayout:
    def __init__(self, shapes: Sequence[Tuple[int, ...]], bucket_elems: int, world_size: int = 1,
                 shard: bool = False, units: "Sequence[Sequence[int]] | None" = None):
        self.shapes = [tuple(int(d) for d in s) for s in shapes]
        self.numels = [int(torch.Size(s).numel()) for s in self.shapes]
        self.world_size = world_size
        bucket_align = ALIGN * (world_size if shard else 1)
        # the atomic units of bucketing, in parameter order (default: one per parameter)
        if units is None:
            units = [[i] for i in range(len(self.shapes))]
        units = [sorted(int(i) for i in u) for u in units if len(u)]
        if sorted(i for u in units for i in u) != list(range(len(self.shapes))):
            raise ValueError("FlatLayout units must partition the parameter indices")
        units.sort(key=lambda u: u[0])
        groups: List[List[int]] = []
        cur: List[int] = []
        cur_n = 0
        for u in reversed(units):
            n = sum(_round_up(self.numels[i], ALIGN) for i in u)
            if cur and cur_n + n > bucket_elems:
                groups.append(cur)
                cur, cur_n = [], 0
            cur.extend(u)
            cur_n += n
        if cur:
            groups.append(cur)
        groups = [sorted(g) for g in reversed(groups)]  # forward order
        self.offsets = [0] * len(self.shapes)
        self.buckets: List[Bucket] = []
        off = 0
        for bi, g in enumerate(groups):
            start = off
            for i in g:
                self.offsets[i] = off
                off += _round_up(self.numels[i], ALIGN)
            length = _round_up(off - start, bucket_align)
            off = start + length
            self.buckets.append(Bucket(bi, start, length, g))
        self.total = max(off, ALIGN)
        self.param_bucket = [0] * len(self.shapes)
        for b in self.buckets:
            for i in b.params:
                self.param_bucket[i] = b.index

    def segments(self) -> List[Tuple[int, Tuple[int, ...]]]:
        return [(o, s) for o, s in zip(self.offsets, self.shapes)]

    def shard_ranges(self, rank: int) -> List[Tuple[int, int]]:
        """(flat start, length) of this rank's shard of every bucket."""
        return [b.shard(rank, self.world_size) for b in self.buckets]

    def shard_numel(self) -> int:
        return sum(b.numel // self.world_size for b in self.buckets)


class FlatParamStore:
    """Owns the flat parameter + gradient buffers; the module's tensors become views into them."""

    def __init__(self, params: List[torch.nn.Parameter], layout: FlatLayout, device: torch.device,
                 dtype: torch.dtype):
        self.params = params
        self.layout = layout
        self.dtype = dtype
        self.param_buf = torch.zeros(layout.total, dtype=dtype, device=device)
        self.grad_buf = torch.zeros(layout.total, dtype=dtype, device=device)
        self.grad_views: List[torch.Tensor] = []
        with torch.no_grad():
            for p, off, n, shape in zip(params, layout.offsets, layout.numels, layout.shapes):
                view = self.param_buf[off:off + n].view(shape)
                view.copy_(p.data.to(device=device, dtype=dtype))
                p.data = view
                self.grad_views.append(self.grad_buf[off:off + n].view(shape))
                p.grad = self.grad_views[-1]

    def user_set_grads(self) -> bool:
        """True if user code replaced some parameter's .grad (not None) since the last rebind."""
        for p, view in zip(self.params, self.grad_views):
            g = p.grad
            if g is not None and g is not view and (g.data_ptr() != view.data_ptr() or g.shape != view.shape):
                return True
        return False

    def grads_state(self) -> int:
        """0: every .grad IS its view; 1: some are None or equivalent views (rebind_grads reattaches
        them); 2: user code set a gradient of its own (``user_set_grads``).  One pass."""
        state = 0
        for p, view in zip(self.params, self.grad_views):
            g = p.grad
            if g is view:
                continue
            if g is not None and (g.data_ptr() != view.data_ptr() or g.shape != view.shape):
                return 2
            state = 1
        return state

    def rebind_grads(self) -> bool:
        """Re-attach gradient views (after user code set ``.grad = None``).  Called every backward:
        the common case (every .grad still IS its cached view) costs one identity test per
        parameter, not a slice per parameter.  Returns True if a user-set gradient was folded in."""
        folded = False
        for p, view in zip(self.params, self.grad_views):
            g = p.grad
            if g is view:
                continue
            if g is not None and g.data_ptr() == view.data_ptr() and g.shape == view.shape:
                continue  # an equivalent view of the same storage
            if g is not None:  # user replaced the grad tensor: fold it back in
                view.copy_(g)
                folded = True
            p.grad = view
        return folded

    def zero_grad(self) -> None:
        self.grad_buf.zero_()
