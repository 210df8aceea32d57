"""Whole-training-step HIP graphs for the engine (DeepSpeed JSON ``"amd": {"hip_graph": true}``).

Reference: one iteration of the loop ``train.py:103-115`` (forward, backward, step).

A data-parallel step of a small model is launch-bound: eager PyTorch issues tens of kernels for
forward + autograd backward, then the gradient collective, the optimizer and the host bookkeeping
(~30 launches + a host sync per step of the reference).  MI355X-first, the step is
captured ONCE per input shape into a HIP graph and replayed:

    zero grads -> loss_fn(*batch) -> autograd backward (grads land in the flat bucket) ->
    [world > 1] gradient collective on the native RCCL communicator, on the capture stream
                (stage 0: all_reduce per bucket; ZeRO-1: reduce_scatter into the shard) ->
    [clipping]  device-side global norm -> clip coefficient (never read on the host) ->
    step counter += 1 on the device -> fused flat Adam (bias corrections from the device counter) ->
    [ZeRO-1]    all_gather of the updated parameter shards

Everything the step reads or writes lives in static buffers (the engine's flat param / grad /
moment buffers, the copied-in batch, the loss output), so a replay is one graph launch.  This is
the HIP-graph replacement for a tracing compiler: no retracing, no Python in the replayed step.

Limits (checked in ``supported``; the engine falls back to eager steps otherwise): CUDA device,
``gradient_accumulation_steps == 1``, no fp16 dynamic loss scaling (its overflow skip is a host
decision), no learning-rate schedule (the lr is baked into the captured Adam launch), and for
``world_size > 1`` the ``nccl`` (RCCL) backend.  Every new input shape first runs ``warmup`` eager
steps of the same body (allocator / library warm-up before capture), then is captured.
"""
from __future__ import annotations

import gc
import weakref
from typing import Callable, Dict, Optional, Tuple

import torch

from ..ops.adam import adam_flat_
from ..parallel import comm


def supported(engine) -> Tuple[bool, str]:
    if engine.device.type != "cuda":
        return False, "HIP graphs need a GPU"
    if engine.gas != 1:
        return False, "gradient_accumulation_steps > 1"
    if engine.loss_scaler is not None:
        return False, "fp16 dynamic loss scaling decides on the host"
    if engine.ds_scheduler is not None or engine.lr_scheduler is not None:
        return False, "a learning-rate schedule changes the captured lr"
    if comm.collectives_on(engine.world_size) and comm.backend_name() != "nccl":
        return False, f"collectives in a graph need RCCL (backend is {comm.backend_name()})"
    return True, ""


def reduce_grads(e, rccl) -> torch.Tensor:
    """What GradReducer does at the boundary, on the current (capture) stream: the optimizer then
    reads ``reducer.reduced`` (the flat bucket, its wire-dtype copy, or the ZeRO shard)."""
    red = e.reducer
    src = red.grad_buf
    if red.comm_buf is not None:
        red.comm_buf.copy_(src)
        src = red.comm_buf
    for bi, b in enumerate(e.layout.buckets):
        view = src[b.start:b.start + b.numel]
        if e.stage >= 1:
            n = b.numel // e.world_size
            out = red.shard_grad[red.shard_offsets[bi]:red.shard_offsets[bi] + n]
            if rccl is not None:
                rccl.reduce_scatter(out, view)
            else:
                out.copy_(view)
        elif rccl is not None:
            rccl.all_reduce(view)
    return red.reduced


def clip_coef(e, rccl, grads: torch.Tensor, scale: float) -> Optional[torch.Tensor]:
    """Device-side global-norm clip coefficient (never read on the host)."""
    clip = e.config.gradient_clipping
    if clip <= 0:
        return None
    sq = grads.float().pow(2).sum() * (scale * scale)
    if e.stage >= 1 and rccl is not None:
        rccl.all_reduce(sq.reshape(1))
    return torch.clamp(clip / (sq.sqrt() + 1e-6), max=1.0).reshape(1).float()


def allgather_params(e, rccl) -> None:
    src = e.param_lp if e.param_lp is not None else e.master
    off = 0
    for b in e.layout.buckets:
        n = b.numel // e.world_size
        out = e.store.param_buf[b.start:b.start + b.numel]
        if rccl is not None:
            rccl.all_gather(out, src[off:off + n])
        else:
            out.copy_(src[off:off + n])
        off += n


def optimizer_tail(e, rccl, step_dev: torch.Tensor, step_ticket: Optional[torch.Tensor] = None) -> None:
    """Everything after the gradients are in the flat bucket, capturable: gradient collective ->
    clip coefficient -> fused flat Adam (which advances the device step counter itself when given
    ``step_ticket``, else one increment launch first) -> [ZeRO-1] parameter all-gather.  The lr and
    Adam constants are baked into the captured launch; ``step_dev`` counts the updates done."""
    grads = reduce_grads(e, rccl)
    scale = 1.0 / e.world_size
    coef = clip_coef(e, rccl, grads, scale)
    g = e.optimizer.param_groups[0]
    if step_ticket is None:
        step_dev.add_(1)
    adam_flat_(e.master, grads, e.exp_avg, e.exp_avg_sq, 1, g["lr"], g["betas"][0], g["betas"][1], g["eps"],
               g["weight_decay"], g["adamw"], grad_scale=scale, grad_scale_dev=coef, param_lp=e.param_lp,
               step_dev=step_dev, step_ticket=step_ticket)
    if e.stage >= 1:
        allgather_params(e, rccl)


class GraphedStep:
    def __init__(self, engine, loss_fn: Callable[..., torch.Tensor], warmup: int = 2, max_graphs: int = 4):
        ok, why = supported(engine)
        if not ok:
            raise RuntimeError(f"hip_graph step unavailable: {why}")
        self.e = engine
        self.loss_fn = loss_fn
        self.warmup = warmup
        self.max_graphs = max_graphs
        self.rccl = None
        if comm.collectives_on(engine.world_size):
            from ..parallel.rccl import RcclComm
            self.rccl = RcclComm(engine.device)
        # the Adam step counter the captured launch reads (the step number of THIS update, 1-based)
        self.step_dev = torch.full((), engine.global_steps - engine.skipped_steps, dtype=torch.int64,
                                   device=engine.device)
        self._step_host = engine.global_steps - engine.skipped_steps  # what step_dev holds (no sync)
        self.lr = engine._sync_client_lr()  # the lr the captured Adam launches carry
        self.step_ticket = torch.zeros((), dtype=torch.int32, device=engine.device)  # (Adam advances step_dev)
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs: Dict[tuple, tuple] = {}  # shape key -> (graph, static inputs, static loss)
        self.seen: Dict[tuple, int] = {}
        self.seeds: Dict[tuple, torch.Tensor] = {}
        self.all_stored: Dict[tuple, bool] = {}  # signature -> its eager step stored every gradient
        from ..ops.loss import _FusedBCEWithLogits, unit_seed
        self._bce_node = _FusedBCEWithLogits._backward_cls
        self._unit = unit_seed(engine.device)  # (made here, outside any capture)
        self.replays = 0
        self.launchers = {}  # key -> _C.DirectLaunch of that signature's graph (graph_module.direct_launcher)
        self.eager_steps = 0
        self._last = None  # (shape, dtype, entry, bound replay) of the last replayed one-tensor signature
        self.failed = ""
        engine.reducer.arm(False)  # the hooks stay silent: the step issues its own collectives

    # ------------------------------------------------------------------ the step body
    def _body(self, *args, key=None, capturing: bool = False) -> torch.Tensor:
        e = self.e
        e.store.rebind_grads()  # .grad views into the flat bucket (host-side binding, no kernel)
        # The bucket is zeroed so the backward may STORE each gradient's first write.  When the
        # eager runs of this signature saw every gradient view stored by the injected kernels, the
        # captured step leaves the zero fill out (one graph node: ~3 us of a ~33 us step): the
        # stores overwrite whatever the bucket holds, and nothing else writes it (the padding
        # between views stays zero from the first fill).
        if not (capturing and self.all_stored.get(key)):
            e.store.grad_buf.zero_()
        loss = self.loss_fn(*args)
        from ..ops.linear import engine_backward
        with engine_backward(grads_zero=True) as stored:  # zeroed just above
            loss.float().backward(self._seed(loss))
        if not capturing:
            self.all_stored[key] = all((v.data_ptr(), v.numel()) in stored for v in e.store.grad_views)
        optimizer_tail(e, self.rccl, self.step_dev, self.step_ticket)
        return loss.detach()

    def _seed(self, loss: torch.Tensor) -> Optional[torch.Tensor]:
        """The backward seed.  The framework's fused BCE (ops/loss.py) only reads its incoming
        gradient and recognises the persistent unit seed: its backward then launches nothing (no
        fill, no multiply node).  Any other loss gets a persistent tensor made only outside capture
        (a tensor from the graph's private pool must not outlive its graph; a capture that finds
        none lets autograd fill its own), re-filled with 1 before every use (one fill node in the
        captured step): a custom Function may edit its grad_output in place."""
        if (loss.grad_fn is not None and type(loss.grad_fn) is self._bce_node and loss.dim() == 0
                and loss.dtype == torch.float32 and not loss.retains_grad):
            return self._unit
        key = (tuple(loss.shape), loss.device)
        seed = self.seeds.get(key)
        if seed is None and not torch.cuda.is_current_stream_capturing():
            seed = self.seeds[key] = torch.ones(loss.shape, dtype=torch.float32, device=loss.device)
        elif seed is not None:
            seed.fill_(1.0)
        return seed

    # ------------------------------------------------------------------ public
    def _sync(self) -> int:
        """Before any step of this callable.  Eager steps of the same engine (``engine(x)`` /
        ``backward`` / ``step``) may have run since the last one: the device step counter the
        captured Adam reads is re-filled from the engine's count when its host mirror disagrees, and
        the client optimizer's lr is read (Engine.step does the same) -- a different lr than the one
        baked into the captured launches drops the graphs (they are recaptured at the new lr).
        Returns the update number this step performs minus one."""
        e = self.e
        want = e.global_steps - e.skipped_steps
        if want != self._step_host:
            self.step_dev.fill_(want)
        lr = e._sync_client_lr()
        if lr != self.lr:
            self.lr = lr
            self._last = None
            self.launchers.clear()
            self.graphs.clear()
        return want

    def _done(self, want: int) -> None:
        e = self.e
        self._step_host = want + 1  # the step's Adam advanced the device counter
        # the flat bucket now holds this step's gradients (the graph leaves them in place): the
        # engine's next eager backward starts from a zeroed buffer
        e._grads_stale = True
        e._finish_graph_step()

    def __call__(self, *args) -> torch.Tensor:
        e = self.e
        want = self._sync()
        last = self._last  # the common case: one tensor argument of last step's signature
        if last is not None and len(args) == 1 and torch.is_tensor(args[0]):
            a = args[0]
            if a.shape == last[0] and a.dtype == last[1]:
                graph, static_in, static_loss = last[2]
                static_in[0].copy_(a, non_blocking=True)
                last[3]()
                self.replays += 1
                self._done(want)
                return static_loss
        key = tuple((tuple(a.shape), a.dtype) if torch.is_tensor(a) else ("py", a) for a in args)
        entry = self.graphs.get(key)
        if entry is None:
            n = self.seen.get(key, 0)
            if n < self.warmup or len(self.graphs) >= self.max_graphs:
                self.seen[key] = n + 1
                loss = self._body(*args, key=key)
                self.eager_steps += 1
                self._done(want)
                return loss
            try:
                entry = self._capture(key, args)
            except Exception as err:  # never lose a step to a capture problem: run it eagerly
                self.failed = f"{type(err).__name__}: {err}"
                from .. import compat
                compat.report_fallback("graph paths", f"whole-step graph capture failed: {self.failed}", e.metrics)
                self.max_graphs = len(self.graphs)
                torch.cuda.synchronize(e.device)
                loss = self._body(*args)
                self.eager_steps += 1
                self._done(want)
                return loss
        graph, static_in, static_loss = entry
        for dst, src in zip(static_in, args):
            if torch.is_tensor(dst):
                dst.copy_(src, non_blocking=True)
        run = self.launchers.get(key) or torch._C._CUDAGraph.replay.__get__(graph)
        run()
        run = self.launchers.get(key) or run  # (a first call may have installed the steady-state launcher)
        if len(args) == 1 and torch.is_tensor(args[0]):
            self._last = (args[0].shape, args[0].dtype, entry, run)
        self.replays += 1
        self._done(want)
        return static_loss

    def _capture(self, key, args):
        static_in = tuple(a.detach().clone() if torch.is_tensor(a) else a for a in args)
        torch.cuda.synchronize(self.e.device)
        graph = torch.cuda.CUDAGraph(keep_graph=True)
        # capture records the launches without running them: the step counter advance is replayed,
        # not double-counted
        gc_on = gc.isenabled()
        try:
            with torch.cuda.graph(graph, pool=self.pool):  # (collects garbage first, then captures)
                gc.disable()  # nothing collected mid-capture (graph_module._capture)
                static_loss = self._body(*static_in, key=key, capturing=True)
        finally:
            if gc_on:
                gc.enable()
        graph.instantiate()
        from .graph_module import direct_launcher, rng_checked  # a short chain of kernels: launched, not replayed
        launcher = direct_launcher(graph)
        if launcher is not None:
            # (first call replays; a graph drawing random numbers stays on replay: rng_checked)
            ref = weakref.ref(self)  # (no cycle through the stored callable: graph_module._setter)
            self.launchers[key] = rng_checked(graph, launcher,
                                              lambda f, key=key: ref() is not None and ref()._install(key, f))
        entry = (graph, static_in, static_loss)
        self.graphs[key] = entry
        return entry

    def _install(self, key, run) -> None:
        """rng_checked's verdict for ``key``'s graph: ``run`` from now on (the fast path re-reads it)."""
        self.launchers[key] = run
        self._last = None

    def close(self) -> None:
        self._last = None
        self.launchers.clear()
        self.graphs.clear()
        if self.rccl is not None:
            self.rccl.close()
            self.rccl = None
