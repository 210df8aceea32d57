"""Bucketed gradient reduction overlapped with backward.

Reference: the gradient all-reduce inside ``model_engine.backward`` (``train.py:113``); SURVEY X6/HC1.

DeepSpeed stage 0 reduces ALL gradients after backward finishes (one 5e8-element bucket, SURVEY
X6): communication never overlaps compute.  Here each bucket (a contiguous slice of the flat
gradient buffer, ``runtime/flat.py``) is launched the moment autograd has accumulated the last
gradient that belongs to it (``register_post_accumulate_grad_hook``), so RCCL moves bucket k over
xGMI while backward computes bucket k-1.  ProcessGroupNCCL runs the collective on its own HIP
stream, ordered after the producing kernels; ``finish()`` joins all of them before the optimizer.

Readiness comes from two places, whichever is first (a parameter counts once per backward):
autograd's post-accumulate hooks, and -- for the framework's fused Linear chains, which are ONE
autograd node for many layers, so their hooks would all fire after the whole chain's backward --
the chain's own per-layer notification right after that layer's weight / bias gradient kernels are
queued (``ops.linear.grad_ready``, wired by ``Engine.backward``).  So bucket L's collective is
queued on the communication stream between layer L's gradient kernels and layer L-1's.

* stage 0: in-place ``all_reduce(SUM)`` of the bucket (or the IPC one-shot kernel for buckets up
  to ``oneshot_max_bytes`` when a validated channel exists: one xGMI hop instead of a ring);
* stage 1/2: ``reduce_scatter_tensor`` of the bucket into this rank's contiguous shard buffer.

The 1/world_size averaging is NOT applied here; it is folded into the fused Adam kernel's
``grad_scale`` (no extra pass over the gradients).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ..runtime.flat import FlatLayout
from . import comm


class GradReducer:
    def __init__(self, grad_buf: torch.Tensor, layout: FlatLayout, stage: int, world_size: int, rank: int,
                 comm_dtype: Optional[torch.dtype] = None, oneshot=None, oneshot_max_bytes: int = 0,
                 debug_sync: bool = False):
        self.grad_buf = grad_buf
        self.layout = layout
        self.stage = stage
        self.world_size = world_size
        self.rank = rank
        self.comm_dtype = comm_dtype or grad_buf.dtype
        self.oneshot = oneshot
        self.oneshot_max_bytes = oneshot_max_bytes
        self.debug_sync = debug_sync
        nb = len(layout.buckets)
        self._param_count = [len(b.params) for b in layout.buckets]
        self._remaining = list(self._param_count)
        self._launched = [False] * nb
        self._ready = [False] * len(layout.shapes)
        self._works: List = []
        self.armed = False
        self._side = None  # the wire-cast stream (comm_buf): the cast runs beside backward, not in it
        self._side_used = False
        # staging buffer when the wire dtype differs from the gradient dtype (e.g. bf16 grads, fp32 comm);
        # a rank that sends nothing (world size 1, collectives not forced) has no wire: the optimizer
        # reads the gradient buffer as it is (no 6 B/param conversion pass, half the optimizer's reads)
        self.comm_buf = (torch.zeros(layout.total, dtype=self.comm_dtype, device=grad_buf.device)
                         if self.comm_dtype != grad_buf.dtype and (stage >= 1 or comm.collectives_on(world_size))
                         else None)
        if stage >= 1:
            self.shard_offsets = []
            off = 0
            for b in layout.buckets:
                self.shard_offsets.append(off)
                off += b.numel // world_size
            self.shard_grad = torch.zeros(off, dtype=self.comm_dtype, device=grad_buf.device)
        else:
            self.shard_offsets = []
            self.shard_grad = None
        self.bytes_reduced = 0

    # the buffer the optimizer reads after finish()
    @property
    def reduced(self) -> torch.Tensor:
        if self.stage >= 1:
            return self.shard_grad
        return self.comm_buf if self.comm_buf is not None else self.grad_buf

    def arm(self, boundary: bool) -> None:
        """Called before backward: only the accumulation-boundary micro-step communicates."""
        self.armed = boundary
        self._remaining = list(self._param_count)
        self._launched = [False] * len(self._launched)
        self._ready = [False] * len(self._ready)
        self._works = []

    @property
    def launches_collectives(self) -> bool:
        """Whether a bucket launch does more than account bytes (worth an early notification)."""
        return self.comm_buf is not None or self.stage >= 1 or comm.collectives_on(self.world_size)

    def on_grad_ready(self, param_index: int) -> None:
        if not self.armed or self._ready[param_index]:
            return
        self._ready[param_index] = True
        b = self.layout.param_bucket[param_index]
        self._remaining[b] -= 1
        if self._remaining[b] == 0:
            self._launch(b)

    def _launch(self, bi: int) -> None:
        if self._launched[bi]:
            return
        self._launched[bi] = True
        b = self.layout.buckets[bi]
        if self.comm_buf is None and self.stage == 0 and not comm.collectives_on(self.world_size):
            # one rank, nothing to send (the optimizer reads grad_buf directly): account only
            self.bytes_reduced += b.numel * self.grad_buf.element_size()
            return
        src = self.grad_buf[b.start:b.start + b.numel]
        side = None
        if self.comm_buf is not None:
            view = self.comm_buf[b.start:b.start + b.numel]
            if src.is_cuda and not torch.cuda.is_current_stream_capturing():
                # the wire cast on a side stream ordered after the producing kernels: the compute
                # stream goes on with the next layer; the collective below is ordered after the cast
                if self._side is None:
                    self._side = torch.cuda.Stream(device=src.device)
                side = self._side
                side.wait_stream(torch.cuda.current_stream(src.device))
                self._side_used = True
                with torch.cuda.stream(side):
                    view.copy_(src)
            else:
                view.copy_(src)
        else:
            view = src
        if side is not None:
            with torch.cuda.stream(side):
                self._issue(bi, b, view)
        else:
            self._issue(bi, b, view)

    def _issue(self, bi: int, b, view: torch.Tensor) -> None:
        self.bytes_reduced += view.numel() * view.element_size()
        if not comm.collectives_on(self.world_size):
            if self.stage >= 1:
                self.shard_grad[self.shard_offsets[bi]:self.shard_offsets[bi] + b.numel].copy_(view)
            return
        if self.debug_sync and view.is_cuda:
            torch.cuda.synchronize()
        if comm.needs_host_staging(view):  # gloo rehearsal of a GPU run: synchronous, via host memory
            if self.stage == 0:
                comm.all_reduce_(view)
            else:
                n = b.numel // self.world_size
                host = view.detach().cpu()
                out = torch.empty(n, dtype=host.dtype)
                dist.reduce_scatter_tensor(out, host)
                self.shard_grad[self.shard_offsets[bi]:self.shard_offsets[bi] + n].copy_(out)
            return
        if self.stage == 0:
            nbytes = view.numel() * view.element_size()
            if (self.oneshot is not None and view.dtype == torch.float32 and nbytes <= self.oneshot_max_bytes
                    and view.numel() <= self.oneshot.stride):
                self.oneshot.allreduce(view, view, 1.0)
            else:
                self._works.append(dist.all_reduce(view, async_op=True))
        else:
            n = b.numel // self.world_size
            out = self.shard_grad[self.shard_offsets[bi]:self.shard_offsets[bi] + n]
            self._works.append(dist.reduce_scatter_tensor(out, view, async_op=True))

    def finish(self) -> None:
        """Launch buckets that received no gradient (unused params), then join all collectives."""
        if not self.armed:
            return
        for bi in reversed(range(len(self._launched))):
            if not self._launched[bi]:
                self._launch(bi)
        for w in self._works:
            w.wait()
        self._works = []
        if self._side_used:  # (the casts, and collectives issued from the side stream)
            torch.cuda.current_stream(self.grad_buf.device).wait_stream(self._side)
            self._side_used = False
        if self.debug_sync and self.grad_buf.is_cuda:
            torch.cuda.synchronize()
        self.armed = False
