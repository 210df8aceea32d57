"""The training engine: a native replacement for the slice of DeepSpeed the reference uses.

Reference call sites (``train.py``): ``deepspeed.initialize`` (87-93), ``engine(x)`` (107),
``engine.backward(loss)`` (113), ``engine.step()`` (114), ``engine.save_checkpoint`` (125),
``engine.train()`` (100) and ``engine.device`` (94).  Semantics kept:

* batch-size derivation + assertion from the JSON config (``config.parse_config``);
* parameters broadcast from rank 0 at construction;
* ``backward`` scales the loss by 1/gradient_accumulation_steps and, at the accumulation boundary,
  reduces gradients across data-parallel ranks (mean);
* ``step`` applies the optimizer at the boundary, zeroes gradients, advances ``global_steps`` and
  logs every ``steps_per_print`` steps;
* DeepSpeed checkpoint layout (``runtime/checkpoint.py``) — plus ``load_checkpoint``.

MI355X-first mechanics (not DeepSpeed's): parameters and gradients are views into flat,
bucket-aligned buffers (``runtime/flat.py``); gradient buckets are reduced by RCCL over xGMI *while
backward runs* (``parallel/reducer.py``); the optimizer is one fused HIP Adam launch over the flat
fp32 master buffer with the 1/world_size average, loss-scale and clip coefficient folded in
(``ops.adam_flat_``); ZeRO-1/2 reduce-scatter gradients into a contiguous shard, update only the
shard, then all-gather parameters per bucket.
"""
from __future__ import annotations

import math
import os
import time
from typing import Any, Dict, Iterable, List, Optional, Tuple

import torch
import torch.distributed as dist

from . import compat
from .config import DSConfig, parse_config
from .ops.adam import adam_flat_
from .ops.linear import engine_backward
from .accelerator import get_accelerator
from .parallel import comm
from .parallel.reducer import GradReducer
from .runtime import checkpoint as ckpt
from .runtime.flat import FlatLayout, FlatParamStore
from .runtime.optim_state import adam_hparams, adam_state_to_flat, flat_to_adam_state
from .runtime.schedules import LossScaler, build_scheduler
from .utils.fault import FaultInjector
from .utils import tracing
from .utils.metrics import MetricsSink, ThroughputTimer

_DTYPES = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}


_DIRECT_KINDS = None


def _direct_node_classes():
    """The autograd node classes of the framework's fused BCE, Linear chain and single Linear
    (identity checks on the direct-backward path instead of class-name strings)."""
    global _DIRECT_KINDS
    if _DIRECT_KINDS is None:
        from .ops.linear import _FusedChainFn, _FusedLinearFn
        from .ops.loss import _FusedBCEWithLogits
        _DIRECT_KINDS = (_FusedBCEWithLogits._backward_cls, _FusedChainFn._backward_cls, _FusedLinearFn._backward_cls)
    return _DIRECT_KINDS


def _torch_mean_bce(node) -> bool:
    """``node`` is torch's binary_cross_entropy_with_logits backward with reduction='mean' and no
    weight / pos_weight: its gradient is the framework loss kernel's (sigmoid(z) - y) / n.  (Only on a
    torch whose node exposes that saved state: compat.features()["torch_bce_node"].)"""
    if type(node).__name__ != "BinaryCrossEntropyWithLogitsBackward0" or not compat.has("torch_bce_node"):
        return False
    try:
        return node._saved_reduction == 1 and node._saved_weight is None and node._saved_pos_weight is None
    except (AttributeError, RuntimeError):  # (saved tensors already freed)
        return False


def _bce_node_class():
    return _direct_node_classes()[0]


class FlatAdamOptimizer:
    """Optimizer facade handed back by ``initialize`` (the engine drives the actual update)."""

    def __init__(self, lr: float, betas, eps: float, weight_decay: float, adamw: bool):
        self.param_groups = [{"lr": lr, "betas": tuple(betas), "eps": eps, "weight_decay": weight_decay,
                              "adamw": adamw}]
        self.engine: Optional["Engine"] = None

    @property
    def lr(self) -> float:
        return self.param_groups[0]["lr"]

    def zero_grad(self, set_to_none: bool = False) -> None:
        if self.engine is not None:
            self.engine.zero_grad()

    def state_dict(self) -> Dict[str, Any]:
        return self.engine.optimizer_state_dict() if self.engine else {}

    def step(self, closure=None):  # DeepSpeed's engine.step() is the supported entry point
        if self.engine is not None:
            self.engine.step()


class Engine:
    def __init__(self, model: torch.nn.Module, config: DSConfig, optimizer=None, lr_scheduler=None,
                 device: Optional[torch.device] = None, model_parameters: Optional[Iterable] = None):
        self.config = config
        self.rank = comm.get_rank()
        self.world_size = comm.get_world_size()
        self.local_rank = comm.rank_info().local_rank
        if device is None:
            device = get_accelerator().device()
        self.device = device
        self.dtype = _DTYPES[config.compute_dtype]
        self.host_cpu = None  # the CPU the host thread is pinned to (amd.pin_host_thread), if any
        if device.type == "cuda" and (config.amd.pin_host_thread
                                      or os.environ.get("DGT_PIN_HOST_THREAD", "0") not in ("", "0")):
            from .accelerator import pin_host_thread
            info = comm.rank_info()
            self.host_cpu = pin_host_thread(info.local_rank, info.local_world_size)
        self.module = model.to(device=device, dtype=self.dtype)
        self.fused_linear_layers = 0
        fused_linear = config.amd.fused_linear
        if fused_linear is None:  # auto: kernel injection (the graphed module captures the kernels too)
            fused_linear = True
        if fused_linear and device.type == "cuda" and self.dtype in (torch.float32, torch.bfloat16):
            # fp32: the small-batch fused Linear kernels (csrc/linear.hip); bf16: the MFMA GEMM chain
            # (ops/mfma_linear.py: gemm.hip + head.hip, no vendor BLAS)
            from .ops.linear import inject_fused_linear
            self.fused_linear_layers = inject_fused_linear(self.module, grad_in_place=True)
        self.stage = config.zero_stage
        self.gas = config.gradient_accumulation_steps
        self.micro_batch = config.train_micro_batch_size_per_gpu
        self.global_steps = 0
        self.global_samples = 0
        self.micro_steps = 0
        self.skipped_steps = 0

        # ---- optimizer hyper-parameters: client torch optimizer, else config, else Adam defaults
        self.client_optimizer = optimizer
        if optimizer is not None and not isinstance(optimizer, FlatAdamOptimizer):
            hp = adam_hparams(optimizer)
        elif config.optimizer is not None:
            o = config.optimizer
            hp = {"lr": o.lr, "betas": o.betas, "eps": o.eps, "weight_decay": o.weight_decay, "adamw": o.adamw}
        else:
            hp = {"lr": 1e-3, "betas": (0.9, 0.999), "eps": 1e-8, "weight_decay": 0.0, "adamw": False}
        self.optimizer = FlatAdamOptimizer(hp["lr"], hp["betas"], hp["eps"], hp["weight_decay"], hp["adamw"])
        self.optimizer.engine = self

        # ---- flat, bucket-aligned parameter / gradient storage
        params = [p for p in (model_parameters if model_parameters is not None else self.module.parameters())
                  if p.requires_grad]
        self.params = list(params)
        self.param_names = self._names(self.params)
        bucket_elems = max(int(config.zero.reduce_bucket_size), 1024)
        # a module's own parameters (a layer's weight and bias) never straddle two buckets: a layer
        # larger than the bucket size is one bucket, bias included (runtime/flat.py units)
        self.layout = FlatLayout([tuple(p.shape) for p in self.params], bucket_elems, self.world_size,
                                 shard=self.stage >= 1, units=self._layer_units(self.params))
        self.store = FlatParamStore(self.params, self.layout, device, self.dtype)
        comm.broadcast_(self.store.param_buf, 0)  # DeepSpeed _broadcast_model

        # ---- fp32 master + moments (full for stage 0, this rank's shard for stage >= 1)
        if self.stage == 0:
            self.master = (self.store.param_buf if self.dtype == torch.float32
                           else self.store.param_buf.float())
            self.param_lp = None if self.dtype == torch.float32 else self.store.param_buf
        else:
            pieces = [self.store.param_buf[s:s + n].float() for s, n in self.layout.shard_ranges(self.rank)]
            self.master = torch.cat(pieces).contiguous()
            self.param_lp = (None if self.dtype == torch.float32
                             else torch.empty(self.master.numel(), dtype=self.dtype, device=device))
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        self._ag_groups = None  # ZeRO: all-gather groups (allgather_bucket_size), built on first use

        # ---- communication
        comm_dtype = None
        if config.communication_data_type:
            comm_dtype = _DTYPES.get(str(config.communication_data_type).replace("float", "fp"), None)
        self.oneshot = None
        if (self.world_size > 1 and device.type == "cuda" and self.stage == 0
                and config.amd.allreduce in ("auto", "oneshot")):
            self.oneshot = self._maybe_oneshot()
        self.reducer = GradReducer(self.store.grad_buf, self.layout, self.stage, self.world_size, self.rank,
                                   comm_dtype=comm_dtype, oneshot=self.oneshot,
                                   oneshot_max_bytes=config.amd.oneshot_max_bytes,
                                   debug_sync=config.amd.debug_sync_streams,
                                   native_comm=self._native_reducer_comm(config))
        # ---- module forward/backward from HIP graphs under the eager API (amd.graph_module)
        self.graph_module = bool(config.amd.graph_module and device.type == "cuda")
        # deferred zeroing needs a writer that STORES gradients (the bf16 MFMA chain, the fp32 fused
        # Linear kernels) and no collective.  Not with graph_module: a graphed backward ADDS into the
        # flat buckets (its captured kernels cannot tell a stale buffer from a fresh one), so after an
        # eager step that deferred its zero fill the next graphed step would add onto stale gradients
        # (ADVICE r4); there the graphed tail zeroes the bucket inside its own replay instead
        self._defer_capable = (device.type == "cuda" and self.world_size == 1 and config.amd.defer_zero_grad
                               and self.dtype in (torch.bfloat16, torch.float32) and self.fused_linear_layers > 0
                               and not self.graph_module)
        self._hooks = []
        self._own_tensor_hooks = set()  # ids of the engine's own tensor hooks (the direct backward runs them)
        self._pindex = {id(p): i for i, p in enumerate(self.params)}
        self.layer_notifications = 0  # parameters reported complete from inside a fused chain's backward
        for i, p in enumerate(self.params):
            self._hooks.append(p.register_post_accumulate_grad_hook(
                lambda _p, i=i: self.reducer.on_grad_ready(i)))
            if self._defer_capable:
                h = p.register_hook(lambda g, p=p: self._before_accumulate(p))
                self._hooks.append(h)
                self._own_tensor_hooks.add(h.id)

        # ---- schedules, loss scaling, logging, fault injection
        self.lr_scheduler = lr_scheduler
        self.ds_scheduler = build_scheduler(config.scheduler.type, config.scheduler.params)
        if self.ds_scheduler is not None:
            self.optimizer.param_groups[0]["lr"] = self.ds_scheduler.step()
        self.loss_scaler = LossScaler(config.loss_scale, config.initial_scale_power) if config.fp16_enabled else None
        self.tput = ThroughputTimer(self.micro_batch * self.world_size, config.steps_per_print)
        self.metrics = MetricsSink.from_env(self.rank)
        self.faults = FaultInjector.from_env(self.rank)
        # the torch internals the graph paths need (compat.py): a torch without them runs eagerly, loudly
        if (self.graph_module or config.amd.hip_graph) and not compat.has("hip_graph"):
            self.graph_module = False
            self.graph_module_reason = compat.features()["hip_graph"]
            compat.report_fallback("graph paths", self.graph_module_reason, self.metrics)
        self._timers: Dict[str, float] = {}
        self._seed_one: Optional[torch.Tensor] = None
        self._grads_dirty = False  # the flat gradient buffer holds something since the last zero_grad
        # Deferred zeroing (one GPU): when the last backward that began on a zeroed buffer STORED every
        # parameter's gradient view (the first writes of the bf16 MFMA chain or of the fp32 fused Linear
        # kernels), the step's zero fill of the flat buffer (a whole-buffer pass: 18.5 us of 800 for
        # the bench MLP; a launch of a host-bound eager step) is skipped -- the next backward
        # overwrites every view anyway.  Should autograd itself accumulate into a view in that
        # backward (a forward that fell back to F.linear, a parameter outside the chains), the view is
        # zeroed just before (a tensor hook runs ahead of AccumulateGrad), and a view nothing writes is
        # zeroed right after the backward (it got no gradient).  So after step() such an engine's .grad
        # views may still hold the last gradients until the next backward: engine.zero_grad() zeroes them.
        self._stored_all = False
        self._zero_deferred = False
        self._deferred_active = False
        self._hook_zeroed = 0  # views zeroed by that hook in the current backward
        self._grad_norm: Optional[torch.Tensor] = None
        # a whole-step graph (graph_step) ran last and left its gradients in the flat bucket: the next
        # eager backward zeroes it first (runtime/graph_step.py GraphedStep._done)
        self._grads_stale = False
        self._boundary_pending = False
        self.training = True
        self.graphed = None
        self.graph_fallback_reason = ""
        self.graph_module_reason = ""
        self._graphed_fwd: Dict[tuple, Any] = {}
        self._runners: List[Any] = []  # every GraphedModule: the copying ones above and their bound ones
        self._view_keys: Optional[list] = None  # _grad_views()
        self._last_graphed = None  # (shape, dtype, requires_grad, GraphedModule) of the last hit
        # graphed tail (runtime/graph_module.py): backward + collective + Adam as one replay when
        # the loss is the framework's own; the step counter Adam reads lives on the device
        self._tail_rccl = None
        self._tail_scratch: Optional[torch.Tensor] = None  # the loss kernel's unused loss output (torch's BCE)
        self._last_torch_bce = None  # the torch BCE node the last direct backward consumed (no second pass)
        self._tail_step_dev: Optional[torch.Tensor] = None
        self._tail_step_host = -1   # what _tail_step_dev holds (host mirror, no sync)
        self._tail_done = False     # backward ran the whole step: step() only does the bookkeeping
        self.tail_steps = 0
        self.direct_backwards = 0   # eager backwards run without the autograd engine (_direct_backward)
        self.tail_reason = ""       # why the graphed tail is not used (empty: in use or not asked)

    # ------------------------------------------------------------------ helpers
    def _layer_units(self, params):
        """Parameter-index groups, one per owning module (its direct parameters), in order."""
        owner = {}
        for m in self.module.modules():
            for p in m.parameters(recurse=False):
                owner.setdefault(id(p), id(m))
        units, index = [], {}
        for i, p in enumerate(params):
            key = owner.get(id(p), ("param", i))
            if key not in index:
                index[key] = len(units)
                units.append([])
            units[index[key]].append(i)
        return units

    def _on_layer_ready(self, p) -> None:
        """A fused chain finished ``p``'s gradient (ops.linear.grad_ready): the reducer may launch its
        bucket now.  A parameter with a user's hook keeps autograd's timing (the hook may still edit
        the gradient before it is accumulated / after)."""
        i = self._pindex.get(id(p))
        if i is None:
            return
        post = p._post_accumulate_grad_hooks
        if (post is not None and len(post) > 1) or any(k not in self._own_tensor_hooks for k in (p._backward_hooks or ())):
            return
        self.layer_notifications += 1
        self.reducer.on_grad_ready(i)

    def _names(self, params):
        lookup = {id(p): n for n, p in self.module.named_parameters()}
        return [lookup.get(id(p), f"param{i}") for i, p in enumerate(params)]

    def _native_reducer_comm(self, config):
        """A native RCCL communicator for the reducer's C++ bucket launcher (parallel/reducer.py), when
        the buckets go over RCCL and there is more than one of them.  Every rank takes the same
        decision (the same config and layout), then all of them bootstrap it together."""
        from .parallel.reducer import _thread_default
        if not (self.device.type == "cuda" and comm.collectives_on(self.world_size) and comm.backend_name() == "nccl"
                and _thread_default() and not config.amd.debug_sync_streams and len(self.layout.buckets) > 1
                and os.environ.get("DGT_REDUCER_NATIVE", "1") != "0"):
            return None
        from .parallel.rccl import RcclComm
        return RcclComm(self.device)

    def _maybe_oneshot(self):
        from .parallel.ipc import IpcChannel, ipc_disabled_by_env
        if ipc_disabled_by_env() or self.world_size > 8:
            return None
        biggest = max(b.numel for b in self.layout.buckets)
        stride = min(biggest, self.config.amd.oneshot_max_bytes // 4)
        try:
            ch = IpcChannel(stride, self.device)
        except Exception:
            return None
        if not ch.selftest():
            ch.close()
            return None
        return ch

    def is_gradient_accumulation_boundary(self) -> bool:
        return (self.micro_steps + 1) % self.gas == 0

    @property
    def lr(self) -> float:
        return self.optimizer.param_groups[0]["lr"]

    def get_lr(self):
        return [self.lr]

    def train(self, mode: bool = True):
        self.training = mode
        self.module.train(mode)
        return self

    def eval(self):
        return self.train(False)

    def zero_grad(self) -> None:
        self.store.zero_grad()
        self._grads_dirty = False
        self._zero_deferred = False
        self._grads_stale = False

    def _sync_client_lr(self) -> float:
        """The lr of the next update: a client torch optimizer's own param group, which the user (or
        their scheduler) may change between steps, else the engine's."""
        g = self.optimizer.param_groups[0]
        c = self.client_optimizer
        if c is not None and not isinstance(c, FlatAdamOptimizer):
            g["lr"] = float(c.param_groups[0]["lr"])
        return g["lr"]

    def _zero_after_step(self) -> None:
        if self._stored_all and self._defer_capable:
            self._zero_deferred = True
            self._grads_dirty = False
        else:
            self.zero_grad()

    def _before_accumulate(self, p) -> None:
        """Autograd is about to ADD into p.grad: in a backward over a deferred (stale) buffer, zero the
        view first unless this backward already wrote it (then the add is the accumulation)."""
        if self._deferred_active and p.grad is not None:
            from .ops.linear import _first_write
            if _first_write(p.grad):
                p.grad.zero_()
                self._hook_zeroed += 1

    def _grad_views(self):
        """(parameter, (data_ptr, numel) of its gradient view): backward rebinds every .grad to its
        flat-bucket view (or an equivalent one) first, so the keys are the store's views' -- built
        once, not per step (the eager step is host-bound)."""
        keys = self._view_keys
        if keys is None:
            keys = self._view_keys = [(p, (v.data_ptr(), v.numel())) for p, v in zip(self.params, self.store.grad_views)]
        return keys

    @property
    def linear_fallbacks(self) -> Dict[str, int]:
        """Calls that left the hand-written Linear kernels for F.linear (vendor BLAS), by reason."""
        from .ops.linear import FALLBACKS
        return dict(FALLBACKS)

    # ------------------------------------------------------------------ forward / backward / step
    def forward(self, *args, **kwargs):
        if args and torch.is_tensor(args[0]) and args[0].dim() > 0:
            # throughput from the REAL micro-batch (DeepSpeed uses the configured one: SURVEY X9)
            self.tput.samples_per_step = int(args[0].shape[0]) * self.world_size
        if self.dtype != torch.float32:
            args = tuple(a.to(self.dtype) if torch.is_tensor(a) and a.is_floating_point() else a for a in args)
        self.tput.start()
        with tracing.range("dgt.forward"):
            if (self.graph_module and self.training and not kwargs and args
                    and (torch.is_tensor(args[0]) if len(args) == 1 else all(torch.is_tensor(a) for a in args))):
                fn = self._graphed_forward(args)
                if fn is not None:
                    if len(args) == 1 and self.config.amd.graph_bind_inputs:
                        b = self._bound_runner(fn, args[0])
                        if b is not None and not b.pending:
                            return b(*args)
                    # a second forward of this signature before the first one's backward runs
                    # eagerly: replaying would overwrite the activations the pending backward needs
                    if not fn.pending:
                        return fn(*args)
            return self.module(*args, **kwargs)

    MAX_GRAPHED_SHAPES = 4
    MAX_BOUND_ADDRESSES = 4
    BIND_BUDGET_BYTES = 1 << 30  # device memory the bound graph pairs of one signature may hold

    def _bound_runner(self, fn, a: torch.Tensor):
        """Graphs that read the input where it lies (``GraphedModule(bind_inputs=True)``): captured
        for an address seen twice in this signature's last 8 calls -- a loader's fresh batch, whose
        block the caching allocator hands back every few steps (the loop variable still holds the
        previous batch while the next one is allocated, so a few addresses take turns) -- and
        replayed whenever the input is there again, which saves the copy into the static input (one
        launch of a host-bound step).  Up to MAX_BOUND_ADDRESSES pairs within BIND_BUDGET_BYTES of
        device memory; a pair unused for 16 calls gives way to a new address.  None: take the
        copying graph."""
        p = a.data_ptr()
        fn.calls += 1
        b = fn.bound.get(p)
        if b is not None:
            if not a.is_contiguous():  # same address, other strides (e.g. a transposed square batch)
                return None
            b.last_use = fn.calls
            return b
        seen, fn.recent = fn.recent, (p,) + fn.recent[:7]
        if seen.count(p) < 2 or fn.bind_failed or a.requires_grad or not a.is_contiguous():
            return None
        if len(fn.bound) >= self.MAX_BOUND_ADDRESSES:
            # addresses of an earlier phase (e.g. before another capture moved the allocator's
            # blocks) make room once unused for a while; bounded, so a churning pattern stops binding
            stale = [q for q, r in fn.bound.items() if not r.pending and fn.calls - r.last_use > 16]
            if not stale:
                return None
            if fn.evictions >= 16:
                fn.bind_failed = "input addresses keep changing"
                return None
            victim = fn.bound.pop(min(stale, key=lambda q: fn.bound[q].last_use))
            self._runners.remove(victim)
            fn.evictions += 1
        if (len(fn.bound) + 1) * fn.footprint > self.BIND_BUDGET_BYTES:
            return None
        from .runtime.graph_module import GraphedModule
        self.store.rebind_grads()
        try:
            # no warmup: the copying pair of this signature already ran it (library handles, workspaces)
            b = GraphedModule(self.module, self.params, (a,), warmup=0, tail=self._tail_callable(), bind_inputs=True)
        except Exception as e:  # keep the copying graph
            fn.bind_failed = f"{type(e).__name__}: {e}"
            return None
        b.last_use = fn.calls
        fn.bound[p] = b
        self._runners.append(b)
        return b

    def _graphed_forward(self, args):
        """The module as a graphed callable for this input signature (``runtime/graph_module.py``):
        forward and backward each replay one HIP graph and the backward graph accumulates straight
        into the flat gradient buckets, so a step costs two graph launches instead of one launch
        per op, autograd node and parameter; the bucket hooks still fire.  Up to
        MAX_GRAPHED_SHAPES signatures are captured; others, and any capture failure, run eagerly."""
        last = self._last_graphed  # the common case: the same single-input signature as last step
        if last is not None and len(args) == 1:
            a = args[0]
            if a.shape == last[0] and a.dtype == last[1] and a.requires_grad == last[2]:
                return last[3]
        from .runtime.graph_module import GraphedModule
        key = tuple((tuple(a.shape), a.dtype, a.requires_grad) for a in args)
        fn = self._graphed_fwd.get(key)
        if fn is not None and len(args) == 1:
            self._last_graphed = (args[0].shape, args[0].dtype, args[0].requires_grad, fn)
        if fn is not None or len(self._graphed_fwd) >= self.MAX_GRAPHED_SHAPES:
            return fn
        self.store.rebind_grads()
        before = torch.cuda.memory_reserved(self.device)
        try:
            fn = GraphedModule(self.module, self.params, args, tail=self._tail_callable())
        except Exception as e:  # data-dependent control flow, host syncs, ...: stay eager
            self.graph_module = False
            self.graph_module_reason = f"capture failed: {type(e).__name__}: {e}"
            compat.report_fallback("graph paths", f"graph_module {self.graph_module_reason}", self.metrics)
            return None
        fn.bound, fn.recent, fn.bind_failed, fn.calls, fn.evictions = {}, (), None, 0, 0
        # what one more graph pair of this signature costs (its pool: activations, outputs)
        fn.footprint = max(0, torch.cuda.memory_reserved(self.device) - before)
        self._graphed_fwd[key] = fn
        self._runners.append(fn)
        return fn

    __call__ = forward

    # ------------------------------------------------------------------ graphed tail
    def _tail_callable(self):
        """The capturable optimizer tail for GraphedModule (None when the config needs host
        decisions between backward and the update: see runtime/graph_step.supported)."""
        if not self.config.amd.graph_tail:
            self.tail_reason = "amd.graph_tail is off"
            return None
        from .runtime.graph_step import optimizer_tail, supported
        ok, why = supported(self)
        if not ok:
            self.tail_reason = why
            return None
        if self._tail_step_dev is None:
            self._tail_step_dev = torch.zeros((), dtype=torch.int64, device=self.device)
            self._tail_ticket = torch.zeros((), dtype=torch.int32, device=self.device)  # (Adam advances the step)
            if comm.collectives_on(self.world_size):
                from .parallel.rccl import RcclComm
                self._tail_rccl = RcclComm(self.device)
        lr = self.optimizer.param_groups[0]["lr"]

        def tail():
            optimizer_tail(self, self._tail_rccl, self._tail_step_dev, self._tail_ticket)
            self.store.grad_buf.zero_()  # consumed: the next step's backward starts from zero
        tail.lr = lr
        return tail

    _VIEW_NODES = ("ViewBackward0", "ReshapeAliasBackward0", "UnsafeViewBackward0", "SqueezeBackward0",
                   "SqueezeBackward1", "SqueezeBackward2", "UnsqueezeBackward0")

    def _tail_runner(self, loss: torch.Tensor):
        """(GraphedModule, dL/dout) when ``loss`` is the framework's fused BCE (``ops/loss.py``) of a
        graphed forward's output, through reshapes / a dtype cast only -- a gradient the engine can
        form without autograd: the BCE kernel already wrote it (d loss / d logits), and with no loss
        scaling and one micro-step the backward seed is 1.  (GraphedModule, (z, y)) for torch's own
        mean BCEWithLogitsLoss of fp32 logits (the reference's criterion): the caller forms dL/dz
        with the framework's loss kernel.  Else None (the autograd path)."""
        node = loss.grad_fn
        if node is None:
            return None
        torch_bce = type(node) is not _bce_node_class()
        if torch_bce and not _torch_mean_bce(node):
            return None
        nxt = node.next_functions  # (logits, targets[, sum_into])
        if len(nxt) < 2 or any(e[0] is not None for e in nxt[1:]):
            return None  # the targets need a gradient too
        cur = nxt[0][0]
        while cur is not None and type(cur).__name__ in self._VIEW_NODES + ("ToCopyBackward0",):
            nn_ = cur.next_functions
            if len(nn_) != 1:
                return None
            cur = nn_[0][0]
        runner = getattr(cur, "runner", None)
        if runner is None or getattr(runner, "bwd_tail", None) is None or not runner.pending:
            return None
        if len(runner.static_out) != 1 or runner.grad_out_idx != [0]:
            return None
        gout = runner.static_gout[0]
        if torch_bce:
            # torch.nn.BCEWithLogitsLoss (the reference's criterion, train.py:96): its dL/dz is formed by
            # the framework's loss kernel straight into the graph's input (see _try_graphed_tail)
            z, y = node._saved_self, node._saved_target
            if (z.dtype != torch.float32 or gout.dtype != torch.float32 or z.numel() != gout.numel()
                    or y.numel() != z.numel() or z.device != gout.device):
                return None
            return runner, (z, y)
        if getattr(node, "freed", True):
            return None
        dz, lp = node.dz, node.lp
        if lp is not None and gout.dtype == lp.dtype:
            dz = lp  # the kernel's once-rounded bf16 copy: a plain copy into the graph's input
        if dz.numel() != gout.numel() or gout.device != dz.device:
            return None
        return runner, dz

    def _try_graphed_tail(self, loss: torch.Tensor, retain_graph: bool = False) -> bool:
        """The graphed tail runs the whole update inside ``backward`` (the captured graph zeroes the
        bucket after Adam): code between backward and step would see zeroed ``.grad``.  So it is
        skipped when the caller keeps the graph for another backward (``retain_graph``) or has set a
        ``.grad`` itself -- both mean gradients are still to be combined before the update."""
        if (retain_graph or not self.graph_module or not self.training or self.gas != 1
                or self.loss_scaler is not None or self._grads_dirty or self.faults.spec is not None
                or self.config.wall_clock_breakdown):
            return False
        grads = self.store.grads_state()
        if grads == 2:  # a user-set .grad
            return False
        found = self._tail_runner(loss)
        if found is None:
            return False
        runner, dz = found
        g = self.optimizer.param_groups[0]
        self._sync_client_lr()
        if g["lr"] != runner.tail_lr:
            self.tail_reason = "the lr changed since the tail was captured"
            return False
        if grads:
            self.store.rebind_grads()
        if self._zero_deferred:  # the last eager step left its gradients in place (deferred zeroing)
            self.store.grad_buf.zero_()
            self._zero_deferred = False
        want = self.global_steps - self.skipped_steps  # the graph adds 1 before its Adam launch
        if self._tail_step_host != want:
            self._tail_step_dev.fill_(want)
        if isinstance(dz, tuple):  # torch's BCE: dL/dz = (sigmoid(z) - y) / n from the fused loss kernel
            z, y = dz
            if self._tail_scratch is None:
                self._tail_scratch = torch.empty((), dtype=torch.float32, device=self.device)
            from .ops import _ext
            _ext.hot().bce_logits(z if z.is_contiguous() else z.contiguous(),
                                  y if (y.dtype == torch.float32 and y.is_contiguous()) else y.float().contiguous(),
                                  self._tail_scratch, runner.static_gout[0], None, None)
        elif dz.data_ptr() != runner.static_gout[0].data_ptr():  # (else the loss kernel wrote it there)
            with torch.no_grad():
                runner.static_gout[0].view(-1).copy_(dz.view(-1))
        with tracing.range("dgt.graphed_tail"):
            runner.tail_replay()
        runner.finish()
        self._tail_step_host = want + 1
        self._tail_done = True
        self.tail_steps += 1
        return True

    def backward(self, loss: torch.Tensor, retain_graph: bool = False) -> torch.Tensor:
        if self._tail_done:
            raise RuntimeError("engine.backward called twice without engine.step() after a graphed-tail step")
        if self._grads_stale:
            self.zero_grad()
        if self._try_graphed_tail(loss, retain_graph):
            return loss
        loss = self.faults.maybe_corrupt_loss(loss, self.global_steps)
        boundary = self.is_gradient_accumulation_boundary()
        if self._zero_deferred and self.store.user_set_grads():
            self.zero_grad()  # a user gradient folds into the buffer below: it must be zero first
        if self.store.rebind_grads():
            self._grads_dirty = True
        self.reducer.arm(boundary and self.training)
        scaled = loss.float()
        if self.gas > 1:
            scaled = scaled / self.gas
        if self.loss_scaler is not None:
            scaled = scaled * self.loss_scaler.scale
        t0 = time.perf_counter() if self.config.wall_clock_breakdown else 0.0
        from_zero, deferred = not self._grads_dirty, self._zero_deferred
        self._zero_deferred = False
        self._deferred_active, self._hook_zeroed = deferred, 0
        # per-layer bucket launches from inside the fused chains, when a launch communicates
        ready = self._on_layer_ready if (self.reducer.armed and self.reducer.launches_collectives) else None
        try:
            with tracing.range("dgt.backward"), engine_backward(grads_zero=from_zero, on_ready=ready) as stored:
                if retain_graph or not self._direct_backward(scaled, loss):
                    scaled.backward(self._backward_seed(scaled, loss), retain_graph=retain_graph)
        finally:
            self._deferred_active = False
        if from_zero:
            views = self._grad_views()
            missing = [p for p, key in views if key not in stored]
            if deferred:
                for p in missing:  # stale from the last step and not written by this backward
                    p.grad.zero_()
            # defer again only when the KERNELS stored every view (an autograd-written view costs a
            # zero launch of its own in a deferred backward)
            self._stored_all = len(views) == len(self.params) and not missing and self._hook_zeroed == 0
        self._grads_dirty = True
        if boundary:
            with tracing.range("dgt.allreduce_wait"):
                self.reducer.finish()
            self._boundary_pending = True
        if self.config.wall_clock_breakdown:
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            self._timers["backward_ms"] = (time.perf_counter() - t0) * 1e3
        return loss

    def _direct_backward(self, scaled: torch.Tensor, loss: torch.Tensor) -> bool:
        """The backward of the engine's own two-node graph without the autograd engine.

        When the loss is the framework's fused BCE (``ops/loss.py``) -- or torch's own mean
        BCEWithLogitsLoss, whose d loss / d logits the framework's loss kernel then forms -- of the
        output of an injected
        Linear chain (``ops/linear.py`` FusedChain / FusedLinear), through reshapes only, and the
        chain's input needs no gradient, the whole graph is two Python backward functions: the BCE's
        (d loss / d logits is already computed: one multiply by the seed) and the chain's (one fused
        backward launch per layer, writing dW / db into the flat bucket).  Calling them directly and
        then running the parameters' post-accumulate hooks (the bucket reducer) the way autograd's
        AccumulateGrad nodes would saves autograd's graph walk and its hand-off to the device's
        worker thread -- most of a host-bound eager step (profiles/r2_engine_host_profile.txt).
        Anything else (another loss, an input that needs a gradient, tensor hooks on a parameter,
        loss scaling or 1/gas nodes) returns False: the caller runs ``scaled.backward``."""
        if (scaled is not loss or not self.config.amd.direct_backward
                or self.device.type != "cuda" or loss.dim() != 0):
            return False
        kinds = _direct_node_classes()
        node = loss.grad_fn
        if node is None:
            return False
        # torch's own mean BCEWithLogitsLoss (the reference's criterion, train.py:96): d loss / d logits
        # comes from the framework's loss kernel, (sigmoid(z) - y) / n, instead of autograd's node
        torch_bce = type(node) is not kinds[0]
        if torch_bce:
            if not _torch_mean_bce(node):
                return False
            z, y = node._saved_self, node._saved_target
            if z.dtype != torch.float32 or not z.is_cuda or y.numel() != z.numel():
                return False
            if node is self._last_torch_bce:
                raise RuntimeError("Trying to backward through the graph a second time: the engine's direct "
                                   "backward already consumed this loss")
        nxt = node.next_functions  # (logits, targets[, sum_into])
        if len(nxt) < 2:
            return False
        for e in nxt[1:]:
            if e[0] is not None:
                return False
        views = []
        cur = nxt[0][0]
        while cur is not None and type(cur) is not kinds[1] and type(cur) is not kinds[2]:
            if type(cur).__name__ not in self._VIEW_NODES + ("ToCopyBackward0",):
                return False
            if len(cur.next_functions) != 1:
                return False
            views.append(cur)
            cur = cur.next_functions[0][0]
        if cur is None:
            return False
        chain = type(cur) is kinds[1]
        edges = cur.next_functions
        if not edges or edges[0][0] is not None:
            return False  # the chain's input wants a gradient too
        leaves = []
        own = self._own_tensor_hooks
        for e in edges[1:]:
            a = e[0]
            if a is None or type(a).__name__ != "AccumulateGrad":
                return False
            p = a.variable
            if p._backward_hooks:
                for k in p._backward_hooks:
                    if k not in own:
                        return False  # a user's tensor hook sees the gradient before accumulation: autograd's job
            leaves.append(p)
        seed = self._unit_seed(loss.device)
        from .ops.loss import direct_backward, release
        prev_grad = torch.is_grad_enabled()
        torch.set_grad_enabled(False)  # grad mode off as under autograd (no create_graph)
        try:
            with direct_backward():
                # the Functions' own backward on their nodes (what BackwardCFunction.apply calls,
                # without its per-call vjp / backward lookup): the unit seed -> the saved d loss /
                # d logits itself, no launch
                if torch_bce:
                    from .ops import _ext
                    g = torch.empty(z.shape, dtype=torch.float32, device=z.device)
                    if self._tail_scratch is None:
                        self._tail_scratch = torch.empty((), dtype=torch.float32, device=self.device)
                    _ext.hot().bce_logits(z if z.is_contiguous() else z.contiguous(),
                                          y if (y.dtype == torch.float32 and y.is_contiguous())
                                          else y.float().contiguous(), self._tail_scratch, g, None, None)
                    self._last_torch_bce = node
                else:
                    g = node._forward_cls.backward(node, seed)
                    g = g[0] if isinstance(g, tuple) else g
                for v in views:  # reshapes / casts back to the chain's output
                    g = v(g)
                    g = g[0] if isinstance(g, tuple) else g
                res = cur._forward_cls.backward(cur, g)
            # what autograd does after a backward that does not retain the graph: the activations and
            # d loss / d logits are freed now (not when the caller drops ``loss``), and a second
            # backward through this graph raises instead of adding the gradients again
            if not torch_bce:
                release(node)
            release(cur)
            # backward outputs -> the tensor inputs the edges belong to (weights, then present biases)
            if chain:
                grads = [gr for j, gr in enumerate(res[3:]) if j % 2 == 0 or cur.has_bias[j // 2]]
            else:
                grads = [res[1]] + ([res[2]] if cur.has_bias else [])
            if len(grads) != len(leaves):
                raise RuntimeError("dgt: direct backward: gradient / parameter count mismatch")
            for p, gr in zip(leaves, grads):
                if gr is None:
                    continue  # written in place into p.grad by the kernels
                if p.grad is None:
                    p.grad = gr.detach()
                else:
                    if p._backward_hooks:
                        self._before_accumulate(p)  # the engine's tensor hook, as autograd would run it
                    p.grad.add_(gr)
        finally:
            torch.set_grad_enabled(prev_grad)
        for p in leaves:  # what AccumulateGrad does after accumulating: the post-accumulate hooks
            hooks = p._post_accumulate_grad_hooks
            if hooks:
                for h in list(hooks.values()):
                    h(p)
        self.direct_backwards += 1
        return True

    def _backward_seed(self, scaled: torch.Tensor, loss: torch.Tensor) -> Optional[torch.Tensor]:
        """A persistent fp32 scalar 1 as the backward seed, saving autograd's per-step ``ones_like``
        fill kernel on a host-bound eager step -- but only when the seed goes into a node the
        engine itself created (the 1/gas division or the loss-scale multiply), whose backward
        reads its incoming gradient without writing it.  A loss the user's code produced directly
        gets autograd's own fresh seed: a custom Function may edit grad_output in place, which
        would corrupt a shared seed for every later step.  The framework's own fused BCE is such a
        node too: its backward only reads the seed (``ops/loss.py``)."""
        own_loss = (scaled is loss and scaled.grad_fn is not None
                    and type(scaled.grad_fn).__name__ == "_FusedBCEWithLogitsBackward")
        if not own_loss and (scaled is loss or scaled.grad_fn is None or scaled.grad_fn is loss.grad_fn):
            return None
        if scaled.dim() != 0 or scaled.dtype != torch.float32 or scaled.retains_grad:
            return None  # (a retained .grad would alias the persistent seed)
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return None
        return self._unit_seed(scaled.device)

    def _unit_seed(self, device: torch.device) -> torch.Tensor:
        seed = self._seed_one
        if seed is None or seed.device != device:
            from .ops.loss import unit_seed
            seed = self._seed_one = unit_seed(device)  # the BCE backward then launches nothing
        return seed

    def _clip_coef(self, grads: torch.Tensor, scale: float) -> Optional[torch.Tensor]:
        clip = self.config.gradient_clipping
        if clip <= 0:
            self._grad_norm = None
            return None
        sq = grads.float().pow(2).sum() * (scale * scale)
        if self.stage >= 1:
            comm.all_reduce_(sq)
        norm = sq.sqrt()
        self._grad_norm = norm
        return torch.clamp(clip / (norm + 1e-6), max=1.0).reshape(1).float()

    def step(self, lr_kwargs=None) -> None:
        self.micro_steps += 1
        for fn in self._runners:  # a forward whose backward never came: its activations are dead
            fn.finish()
        if self._tail_done:  # the graphed tail already reduced, clipped, updated and zeroed
            self._tail_done = False
            self._finish_step(skipped=False, zero=False)
            return
        if not self._boundary_pending:
            return
        self._boundary_pending = False
        t0 = time.perf_counter() if self.config.wall_clock_breakdown else 0.0
        grads = self.reducer.reduced
        scale = 1.0 / self.world_size
        if self.loss_scaler is not None:
            scale /= self.loss_scaler.scale
            overflow = not bool(torch.isfinite(grads).all().item())
            if self.stage >= 1 and comm.collectives_on(self.world_size):
                overflow = comm.all_reduce_max(float(overflow), self.device) > 0
            self.loss_scaler.update(overflow)
            if overflow:
                self.skipped_steps += 1
                self._finish_step(skipped=True)
                return
        self._sync_client_lr()
        coef = self._clip_coef(grads, scale)
        g = self.optimizer.param_groups[0]
        with tracing.range("dgt.adam"):
            adam_flat_(self.master, grads, self.exp_avg, self.exp_avg_sq, self.global_steps + 1 - self.skipped_steps,
                       g["lr"], g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"], g["adamw"],
                       grad_scale=scale, grad_scale_dev=coef, param_lp=self.param_lp)
        if self.stage >= 1:
            self._allgather_params()
        self._finish_step(skipped=False)
        if self.config.wall_clock_breakdown:
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            self._timers["step_ms"] = (time.perf_counter() - t0) * 1e3

    def _allgather_group_plan(self):
        """Reduce buckets grouped into all-gather groups of at most ``allgather_bucket_size``
        elements (DeepSpeed's knob; default 8M elements = 32 MiB of fp32).  Each group goes out as ONE
        coalesced RCCL launch (a group call: every rank's shards of every bucket of the group in
        flight together), so on an 8 x MI355X node a group keeps the 7 xGMI links of every GPU busy
        for tens of microseconds instead of paying one collective's latency per small bucket."""
        cap = max(int(self.config.zero.allgather_bucket_size), 1)
        groups, cur, n = [], [], 0
        for i, b in enumerate(self.layout.buckets):
            if cur and n + b.numel > cap:
                groups.append(cur)
                cur, n = [], 0
            cur.append(i)
            n += b.numel
        if cur:
            groups.append(cur)
        return groups

    def _allgather_params(self) -> None:
        src = self.param_lp if self.param_lp is not None else self.master
        on = comm.collectives_on(self.world_size)
        if self._ag_groups is None:
            self._ag_groups = self._allgather_group_plan()
        pieces, off = [], 0
        for b in self.layout.buckets:
            n = b.numel // self.world_size
            pieces.append((self.store.param_buf[b.start:b.start + b.numel], src[off:off + n]))
            off += n
        works = []
        coalesce = on and comm.backend_name() == "nccl" and hasattr(dist, "_coalescing_manager")
        for group in self._ag_groups:
            if not on:
                for i in group:
                    pieces[i][0].copy_(pieces[i][1])
            elif comm.needs_host_staging(pieces[group[0]][0]):
                for i in group:
                    out, piece = pieces[i]
                    host = torch.empty(out.numel(), dtype=piece.dtype)
                    dist.all_gather_into_tensor(host, piece.detach().cpu())
                    out.copy_(host)
            elif coalesce:
                with dist._coalescing_manager(device=self.device, async_ops=True) as cm:
                    for i in group:
                        dist.all_gather_into_tensor(pieces[i][0], pieces[i][1])
                works.append(cm)
            else:
                works.extend(dist.all_gather_into_tensor(pieces[i][0], pieces[i][1], async_op=True) for i in group)
        for w in works:
            w.wait()

    # ------------------------------------------------------------------ whole-step HIP graphs
    def graph_step(self, loss_fn, warmup: int = 2):
        """A callable ``step(*batch) -> loss`` running forward + backward + gradient collective +
        optimizer as one replayed HIP graph per input shape (``runtime/graph_step.py``).  Where a
        graph cannot represent the configuration it returns the equivalent eager closure."""
        from .runtime.graph_step import GraphedStep, supported
        ok, why = supported(self)
        if ok and not compat.has("hip_graph"):
            ok, why = False, compat.features()["hip_graph"]
        if ok:
            self.graphed = GraphedStep(self, loss_fn, warmup=warmup)
            return self.graphed
        self.graph_fallback_reason = why
        compat.report_fallback("graph paths", f"whole-step graph: {why}", self.metrics)

        def eager(*args):
            loss = loss_fn(*args)
            self.backward(loss)
            self.step()
            return loss.detach()
        return eager

    def _finish_graph_step(self) -> None:
        self.micro_steps += 1
        self.tput.start()
        self._finish_step(skipped=False, zero=False)

    def _finish_step(self, skipped: bool, zero: bool = True) -> None:
        if zero:
            self._zero_after_step()
        self.global_steps += 1
        self.global_samples += self.config.train_batch_size
        if self.lr_scheduler is not None and not skipped:
            self.lr_scheduler.step()
        if self.ds_scheduler is not None and not skipped:
            self.optimizer.param_groups[0]["lr"] = self.ds_scheduler.step()
        self.tput.stop(self.global_steps)
        if self.global_steps % self.config.steps_per_print == 0 and self.rank == 0:
            g = self.optimizer.param_groups[0]
            msg = (f"[Rank 0] step={self.global_steps}, skipped={self.skipped_steps}, lr={[g['lr']]}, "
                   f"mom={[tuple(g['betas'])]}")
            sps = self.tput.samples_per_sec()
            if sps:
                msg += f", samples/sec={sps:.1f}"
            if self._timers:
                msg += ", " + ", ".join(f"{k}={v:.3f}" for k, v in self._timers.items())
            if os.environ.get("DGT_QUIET", "0") == "0":
                print(msg, flush=True)
        if self.metrics.enabled:  # (no per-step record built for a disabled sink: host-bound eager steps)
            self.metrics.log({"step": self.global_steps, "lr": self.lr, "skipped": int(skipped),
                              "samples_per_sec": self.tput.samples_per_sec(),
                              "comm_bytes": self.reducer.bytes_reduced, **self._timers})
        if self.faults.spec is not None:
            self.faults.maybe_fire(self.global_steps)

    # ------------------------------------------------------------------ state
    def module_state_dict(self) -> Dict[str, torch.Tensor]:
        return {k: v.detach().cpu().clone() for k, v in self.module.state_dict().items()}

    def optimizer_state_dict(self) -> Dict[str, Any]:
        g = self.optimizer.param_groups[0]
        if self.stage >= 1:
            raise RuntimeError("ZeRO optimizer state is sharded; see the zero_pp_rank_* checkpoint files")
        st = flat_to_adam_state(self.exp_avg, self.exp_avg_sq, self.layout.segments(), self.global_steps
                                - self.skipped_steps, g["lr"], g["betas"], g["eps"], g["weight_decay"], g["adamw"])
        if self.master.data_ptr() != self.store.param_buf.data_ptr():
            # bf16 / fp16 run: the module holds the low-precision copy, so the fp32 masters travel with
            # the optimizer state (DeepSpeed's bf16 optimizer keeps its fp32 groups there too) --
            # without them a resumed run restarts from rounded weights and drifts off the original
            st["single_partition_of_fp32_groups"] = [self.master.detach().cpu().clone()]
            # where each named parameter sits in that flat master (zero_to_fp32 unflattens it)
            st["fp32_param_names"] = list(self.param_names)
            st["fp32_param_segments"] = [(int(o), tuple(int(d) for d in s)) for o, s in self.layout.segments()]
        return st

    def _zero_shard_state(self) -> Dict[str, Any]:
        g = self.optimizer.param_groups[0]
        return {
            "zero_stage": self.stage,
            "partition_rank": self.rank,
            "partition_world_size": self.world_size,
            "buckets": [[b.start, b.numel] for b in self.layout.buckets],
            "offsets": list(self.layout.offsets),
            "shapes": [list(s) for s in self.layout.shapes],
            "names": list(self.param_names),
            "total": self.layout.total,
            "fp32_flat": self.master.detach().cpu().clone(),
            "exp_avg": self.exp_avg.detach().cpu().clone(),
            "exp_avg_sq": self.exp_avg_sq.detach().cpu().clone(),
            "step": self.global_steps - self.skipped_steps,
            "param_groups": [{"lr": g["lr"], "betas": list(g["betas"]), "eps": g["eps"],
                              "weight_decay": g["weight_decay"], "adamw": g["adamw"]}],
        }

    def save_checkpoint(self, save_dir: str, tag: Optional[str] = None, client_state: Optional[dict] = None,
                        save_latest: bool = True) -> str:
        extra = {"global_samples": self.global_samples, "skipped_steps": self.skipped_steps,
                 "dp_world_size": self.world_size, "client_state": client_state or {},
                 "lr_scheduler": (self.ds_scheduler.state_dict() if self.ds_scheduler is not None else
                                  (self.lr_scheduler.state_dict() if self.lr_scheduler is not None else None))}
        if self.loss_scaler is not None:
            extra["client_state"] = dict(extra["client_state"], _loss_scaler=self.loss_scaler.state_dict())
        return ckpt.save(save_dir, tag, self.global_steps, self.module_state_dict(),
                         None if self.stage >= 1 else self.optimizer_state_dict(), extra, self.config.to_dict(),
                         zero_shard=self._zero_shard_state() if self.stage >= 1 else None,
                         save_latest=save_latest)

    def load_checkpoint(self, load_dir: str, tag: Optional[str] = None, load_optimizer_states: bool = True,
                        load_lr_scheduler_states: bool = True) -> Tuple[Optional[str], Optional[dict]]:
        path, states, shard = ckpt.load(load_dir, tag)
        if states is None:
            return None, None
        sd = states["module"]
        self.module.load_state_dict({k: v.to(self.dtype) if v.is_floating_point() else v for k, v in sd.items()})
        self.global_steps = int(states.get("global_steps", 0))
        self.global_samples = int(states.get("global_samples", 0))
        self.skipped_steps = int(states.get("skipped_steps", 0))
        if self.stage == 0:
            if self.master.data_ptr() != self.store.param_buf.data_ptr():
                fp32 = (states.get("optimizer") or {}).get("single_partition_of_fp32_groups")
                if fp32 and fp32[0].numel() == self.master.numel():
                    self.master.copy_(fp32[0].to(self.master))
                else:  # a checkpoint without masters (fp32 run, or another writer): start from the module
                    self.master.copy_(self.store.param_buf.float())
            if load_optimizer_states and states.get("optimizer"):
                adam_state_to_flat(states["optimizer"], self.exp_avg, self.exp_avg_sq, self.layout.segments())
        else:
            if shard is None:
                raise FileNotFoundError(f"missing ZeRO shard for rank {self.rank} under {path}")
            if int(shard["partition_world_size"]) != self.world_size or int(shard["total"]) != self.layout.total:
                raise RuntimeError("ZeRO checkpoint was written with a different world size / layout; "
                                   "consolidate it with zero_to_fp32.py and load the fp32 weights instead")
            self.master.copy_(shard["fp32_flat"].to(self.master))
            if load_optimizer_states:
                self.exp_avg.copy_(shard["exp_avg"].to(self.exp_avg))
                self.exp_avg_sq.copy_(shard["exp_avg_sq"].to(self.exp_avg_sq))
            if self.param_lp is not None:
                self.param_lp.copy_(self.master)
            self._allgather_params()
        if load_lr_scheduler_states and states.get("lr_scheduler") is not None:
            if self.ds_scheduler is not None:
                self.ds_scheduler.load_state_dict(states["lr_scheduler"])
                self.optimizer.param_groups[0]["lr"] = self.ds_scheduler.get_lr()
            elif self.lr_scheduler is not None:
                self.lr_scheduler.load_state_dict(states["lr_scheduler"])
        cs = dict(states.get("client_state") or {})
        if self.loss_scaler is not None and "_loss_scaler" in cs:
            self.loss_scaler.load_state_dict(cs.pop("_loss_scaler"))
        return path, cs

    def close(self) -> None:
        if self.graphed is not None:
            self.graphed.close()
            self.graphed = None
        self._graphed_fwd.clear()  # graph_module: the captured graphs and their memory pools
        self._runners = []
        self._last_graphed = None
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.reducer.close()
        if self.oneshot is not None:
            self.oneshot.close()
            self.oneshot = None
        self.metrics.close()


def initialize(args=None, model: Optional[torch.nn.Module] = None, optimizer=None, model_parameters=None,
               training_data=None, lr_scheduler=None, config=None, config_params=None, collate_fn=None,
               dist_init_required: Optional[bool] = None):
    """DeepSpeed-compatible ``initialize`` -> ``(engine, optimizer, training_dataloader, lr_scheduler)``.

    ``config`` (or ``config_params``) is a dict or a JSON path.  ``args`` is accepted for call
    compatibility (the reference passes its config dict there too) and is otherwise
    used only for ``args.deepspeed_config``.
    """
    if model is None:
        raise ValueError("initialize() needs a model")
    cfg_src = config if config is not None else config_params
    if cfg_src is None and args is not None and getattr(args, "deepspeed_config", None):
        cfg_src = args.deepspeed_config
    if not comm.is_initialized() and dist_init_required is not False:
        comm.init_distributed()
    cfg = parse_config(cfg_src, comm.get_world_size())
    engine = Engine(model, cfg, optimizer=optimizer, lr_scheduler=lr_scheduler, model_parameters=model_parameters)
    loader = None
    if training_data is not None:
        from torch.utils.data import DataLoader, DistributedSampler
        sampler = DistributedSampler(training_data, num_replicas=comm.get_world_size(), rank=comm.get_rank())
        loader = DataLoader(training_data, batch_size=cfg.train_micro_batch_size_per_gpu, sampler=sampler,
                            collate_fn=collate_fn)
    return engine, engine.optimizer, loader, (engine.ds_scheduler or lr_scheduler)
