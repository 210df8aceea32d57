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

Launching a bucket costs the host far more than a kernel launch (ProcessGroupNCCL's stream / event
bookkeeping, RCCL's enqueue, the wire cast): done on the thread that enqueues backward, it left the
compute stream idle between layers (profiles/r6_engine_overlap_trace_v1.txt: 60-180 us gaps per
bucket).  So on the GPU the reducer hands each ready bucket to ONE launcher thread: the backward
thread only records a HIP event on its stream (the point the bucket's gradients are complete) and
queues (bucket, event); the launcher makes its side stream wait for that event, casts to the wire
dtype there and issues the collective from it.  One thread issues every collective, in notification
order, so all ranks issue the same sequence; ``finish()`` drains the queue before it joins the
collectives.  (``DGT_REDUCER_THREAD=0``: launches on the backward thread.)

With the RCCL backend that launcher is NATIVE (``csrc/bucket_launcher.cpp``, given a native
communicator, ``parallel/rccl.py``): a C++ thread that never takes the interpreter lock waits for the
event on its side stream, widens bf16 gradients onto the fp32 wire buffer there and enqueues
ncclAllReduce / ncclReduceScatter; the backward thread's whole cost of a bucket is one event record
and a queue push.  Buckets small enough for the IPC one-shot all-reduce stay on the Python path
(inline).  Elsewhere (gloo, other wire dtypes) a Python launcher thread does the same.

* stage 0: in-place ``all_reduce(SUM)`` of the bucket (or the IPC one-shot kernel for buckets up
  to ``oneshot_max_bytes`` when a validated channel exists: one xGMI hop instead of a ring);
* stage 1/2: ``reduce_scatter_tensor`` of the bucket into this rank's contiguous shard buffer.

The 1/world_size averaging is NOT applied here; it is folded into the fused Adam kernel's
``grad_scale`` (no extra pass over the gradients).
"""
from __future__ import annotations

import os
import queue
import threading
import weakref
from typing import List, Optional

import torch
import torch.distributed as dist

from ..runtime.flat import FlatLayout
from . import comm


def _thread_default() -> bool:
    return os.environ.get("DGT_REDUCER_THREAD", "1") not in ("", "0", "false", "False")


class GradReducer:
    def __init__(self, grad_buf: torch.Tensor, layout: FlatLayout, stage: int, world_size: int, rank: int,
                 comm_dtype: Optional[torch.dtype] = None, oneshot=None, oneshot_max_bytes: int = 0,
                 debug_sync: bool = False, launch_thread: Optional[bool] = None, native_comm=None):
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
        self._side = None  # the stream the casts and collectives are issued from (GPU)
        self.side_concurrent = None  # whether that stream was measured to run beside the compute stream
        self._side_used = False
        # the launcher thread (module docstring): GPU tensors with more than one bucket by default (a
        # single bucket is launched at the end of backward anyway: a hand-off would only add the
        # thread's wake-up to the step); a test may force it on the CPU
        self.launch_thread = ((_thread_default() and grad_buf.is_cuda and nb > 1) if launch_thread is None
                              else launch_thread)
        self._q: Optional[queue.Queue] = None
        self._worker: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None
        self.thread_launches = 0
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
        # the native launcher (module docstring) for every bucket the one-shot path does not take
        self.native = None
        self._native_comm = native_comm
        self._inline = set()
        if native_comm is not None and self.launch_thread and not debug_sync:
            self._native_setup(native_comm)

    def _oneshot_bucket(self, bi: int) -> bool:
        b = self.layout.buckets[bi]
        return (self.stage == 0 and self.oneshot is not None and self.comm_dtype == torch.float32
                and b.numel * 4 <= self.oneshot_max_bytes and b.numel <= self.oneshot.stride)

    def _native_setup(self, rc) -> None:
        wire = self.comm_buf if self.comm_buf is not None else self.grad_buf
        if not (wire is self.grad_buf or (self.grad_buf.dtype == torch.bfloat16 and wire.dtype == torch.float32)):
            return
        from ..ops._ext import fast, require
        ops = require()
        nb = len(self.layout.buckets)
        self._inline = {bi for bi in range(nb) if self._oneshot_bucket(bi)}
        offs = torch.tensor([b.start for b in self.layout.buckets], dtype=torch.int64)
        nums = torch.tensor([b.numel for b in self.layout.buckets], dtype=torch.int64)
        soffs = torch.tensor(self.shard_offsets if self.stage >= 1 else [0] * nb, dtype=torch.int64)
        # the launcher issues on the reducer's side stream: normal priority, on a hardware queue other
        # than the compute stream's (accelerator.concurrent_stream; csrc/bucket_launcher.cpp)
        side = self._side_stream().cuda_stream
        self.native = int(ops.bucket_launcher_create(rc.handle, self.grad_buf, wire, self.shard_grad, offs, nums,
                                                     soffs, self.stage, self.world_size, int(side)))
        self._submit = fast().bucket_launcher_submit
        self._native_finish = ops.bucket_launcher_finish
        self._native_launched = ops.bucket_launcher_launched
        self._native_pending = False

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

    # ------------------------------------------------------------------ launching a bucket
    def _launch(self, bi: int) -> None:
        if self._launched[bi]:
            return
        self._launched[bi] = True
        b = self.layout.buckets[bi]
        if self.comm_buf is None and self.stage == 0 and not comm.collectives_on(self.world_size):
            # one rank, nothing to send (the optimizer reads grad_buf directly): account only
            self.bytes_reduced += b.numel * self.grad_buf.element_size()
            return
        cuda = self.grad_buf.is_cuda
        capturing = cuda and torch.cuda.is_current_stream_capturing()
        if self.native is not None and not capturing and bi not in self._inline:
            self.bytes_reduced += b.numel * (self.comm_buf if self.comm_buf is not None else self.grad_buf).element_size()
            self._submit(self.native, bi)  # one event record + a queue push; the C++ thread does the rest
            self._native_pending = True
            return
        staged = comm.collectives_on(self.world_size) and comm.needs_host_staging(self.grad_buf)
        if self.launch_thread and not capturing and not self.debug_sync and not staged:
            ev = None
            if cuda:  # the point on the producing stream where this bucket's gradients are complete
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.grad_buf.device))
            if self._q is None:
                self._start_worker()
            self._q.put((bi, ev))
            return
        # inline: a wire cast still goes to the side stream (beside backward); an in-place collective
        # is issued from the current stream as it is (ProcessGroupNCCL orders its stream after it)
        side_cast = cuda and not capturing and self.comm_buf is not None
        self._launch_now(bi, torch.cuda.current_stream(self.grad_buf.device) if side_cast else None)

    def _side_stream(self):
        if self._side is None:
            # a stream on a hardware queue other than the compute stream's (accelerator.concurrent_stream):
            # on a shared queue the casts and collectives would run in turn with backward, not beside it
            from ..accelerator import concurrent_stream
            self._side, self.side_concurrent = concurrent_stream(self.grad_buf.device)
        return self._side

    def _launch_now(self, bi: int, after) -> None:
        """Cast (if the wire dtype differs) and issue bucket ``bi``'s collective.  ``after``: a stream
        or an event the side stream first waits for (GPU, not capturing); None: the current stream."""
        b = self.layout.buckets[bi]
        src = self.grad_buf[b.start:b.start + b.numel]
        view = src if self.comm_buf is None else self.comm_buf[b.start:b.start + b.numel]
        if after is None:
            if view is not src:
                view.copy_(src)
            self._issue(bi, b, view)
            return
        side = self._side_stream()
        if isinstance(after, torch.cuda.Event):
            side.wait_event(after)
        else:
            side.wait_stream(after)
        self._side_used = True
        with torch.cuda.stream(side):
            if view is not src:
                view.copy_(src)  # the wire cast beside backward, not in it
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

    # ------------------------------------------------------------------ the launcher thread
    def _start_worker(self) -> None:
        # the thread holds the reducer weakly (no reference cycle through its target), and a reducer
        # that is collected without close() stops it through the finalizer's sentinel
        self._q = q = queue.Queue()
        self._worker = threading.Thread(target=GradReducer._work_loop, args=(weakref.ref(self), q, self.grad_buf.device),
                                        daemon=True, name="dgt-reducer")
        weakref.finalize(self, q.put, None)
        self._worker.start()

    @staticmethod
    def _work_loop(ref, q, dev) -> None:
        if dev.type == "cuda":
            torch.cuda.set_device(dev)  # (the current device is per thread)
        while True:
            item = q.get()
            r = None
            try:
                if item is None:
                    return
                r = ref()
                if r is None:
                    return
                if r._error is None:
                    bi, ev = item
                    r._launch_now(bi, ev)
                    r.thread_launches += 1
            except BaseException as e:  # noqa: BLE001 -- re-raised by finish() on the backward thread
                if r is not None:
                    r._error = e
            finally:
                r = None
                q.task_done()

    def _drain(self) -> None:
        if self._q is not None:
            self._q.join()
            if self._error is not None:
                err, self._error = self._error, None
                raise RuntimeError(f"gradient bucket launch failed on the launcher thread: {err}") from err

    def finish(self) -> None:
        """Launch buckets that received no gradient (unused params), then join all collectives."""
        if not self.armed:
            return
        for bi in reversed(range(len(self._launched))):
            if not self._launched[bi]:
                self._launch(bi)
        self._drain()
        if self.native is not None and self._native_pending:
            self._native_finish(self.native)  # the current stream now waits for the native collectives
            self._native_pending = False
        for w in self._works:
            w.wait()
        self._works = []
        if self._side_used:  # (the casts, and collectives issued from the side stream)
            torch.cuda.current_stream(self.grad_buf.device).wait_stream(self._side)
            self._side_used = False
        if self.debug_sync and self.grad_buf.is_cuda:
            torch.cuda.synchronize()
        self.armed = False

    @property
    def native_launches(self) -> int:
        return int(self._native_launched(self.native)) if self.native is not None else 0

    def close(self) -> None:
        """Stop the launcher threads (after a last drain)."""
        if self.native is not None:
            from ..ops._ext import require
            h, self.native = self.native, None
            try:
                if self._native_pending:
                    self._native_finish(h)
            finally:
                require().bucket_launcher_destroy(h)
        if self._native_comm is not None:
            self._native_comm.close()
            self._native_comm = None
        if self._q is not None:
            try:
                self._drain()
            finally:
                self._q.put(None)
                self._worker.join(timeout=10.0)
                self._q, self._worker = None, None
