"""DeepSpeed-compatible JSON configuration.

The reference builds its engine config in code (``train.py:78-83``)::

    {"train_batch_size": 64, "gradient_accumulation_steps": 1,
     "fp16": {"enabled": False}, "zero_optimization": {"stage": 0}}

and hands it to ``deepspeed.initialize``.  DeepSpeed derives the micro batch
from it and asserts ``train_batch_size == micro * gas * world_size`` (SURVEY
Q2/Q3).  This module parses the same schema (dict or JSON path), applies the
same derivation/assertion with a clearer message, and adds the MI355X-specific
knobs under an ``"amd"`` section (all optional).

Byte-size defaults are chosen for xGMI, not NVSwitch: a ring collective on an
8x MI355X node is bounded by ONE ~153 GB/s link per GPU, so buckets of a few
tens of MB keep each link busy for ~100+ us per collective while still being
small enough to overlap with backward.  DeepSpeed's 5e8-element default would
serialize all communication after backward.
"""
from __future__ import annotations

import copy
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, Optional, Union

# the reference config verbatim (train.py:78-83)
REFERENCE_DS_CONFIG: Dict[str, Any] = {
    "train_batch_size": 64,
    "gradient_accumulation_steps": 1,
    "fp16": {"enabled": False},
    "zero_optimization": {"stage": 0},
}

# Default gradient bucket: 32 MiB (8M fp32 elements).  DeepSpeed's default (5e8 elements = 2 GB)
# puts the whole model in one bucket, so nothing overlaps backward.  On an 8 x MI355X node a ring
# all-reduce is bound by ONE xGMI link per hop (~153 GB/s) and RCCL splits a message
# across its channels: 32 MiB gives every channel multi-MB pieces (near the bus-bandwidth plateau of
# the rccl_perf sweep) while the first bucket still leaves backward after ~1/N of its work, so the
# remaining buckets overlap the rest of backward.  Buckets at or below ``amd.oneshot_max_bytes``
# (256 KiB) take the one-hop IPC exchange instead, where latency, not link bandwidth, rules.
DEFAULT_BUCKET_BYTES = 32 * 1024 * 1024


class ConfigError(ValueError):
    pass


@dataclass
class ZeroConfig:
    stage: int = 0
    reduce_bucket_size: int = DEFAULT_BUCKET_BYTES // 4   # elements (DeepSpeed unit)
    allgather_bucket_size: int = DEFAULT_BUCKET_BYTES // 4
    overlap_comm: bool = True
    contiguous_gradients: bool = True
    reduce_scatter: bool = True


@dataclass
class OptimizerConfig:
    type: str = "Adam"
    lr: float = 1e-3
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.0
    adamw: bool = False


@dataclass
class SchedulerConfig:
    type: Optional[str] = None
    params: Dict[str, Any] = field(default_factory=dict)


@dataclass
class AMDConfig:
    # "auto": one-shot xGMI all-reduce for small buckets, RCCL for the rest
    allreduce: str = "auto"
    # messages up to this size use the IPC one-shot path when it is available
    oneshot_max_bytes: int = 256 * 1024
    hip_graph: bool = False
    # extra sync between comm and compute streams: validates overlap logic
    debug_sync_streams: bool = False
    # kernel injection: nn.Linear (+ following nn.ReLU) -> hand-written HIP kernels (ops/linear.py:
    # fp32 small-batch fused launches or the fp32 MFMA GEMM; bf16 the MFMA chain).  None = auto: on
    # for a GPU engine (torch's F.linear costs ~37 us of host dispatch per call on ROCm at the
    # reference's shapes: eager engine 2,450 -> 4,300 it/s, profiles/r2_engine_host_profile.txt);
    # with graph_module the graphs capture these kernels
    fused_linear: Optional[bool] = None
    # the module's forward and backward replayed from HIP graphs (one pair per input shape) under
    # the ordinary engine(x) / engine.backward(loss) / engine.step() calls (engine.py)
    graph_module: bool = False
    # with graph_module: when the loss is the framework's fused BCE of the graphed output,
    # engine.backward replays backward + gradient collective + clip + Adam as ONE graph and
    # engine.step() only does the bookkeeping (so parameters are updated when backward returns)
    graph_tail: bool = True
    # with graph_module: an input that arrives at the same address step after step (a loader's
    # fresh batch, recycled by the caching allocator) gets graphs that read it in place -- no copy
    # into a static input (up to 2 addresses per input shape; others take the copying graph)
    graph_bind_inputs: bool = True
    # eager: engine.backward runs the backward of its own loss -> Linear-chain graph (fused BCE of an
    # injected chain's output) by calling the two backward functions directly, without the autograd
    # engine; any other graph goes through autograd (engine.py Engine._direct_backward)
    direct_backward: bool = True
    # one GPU, injected kernels that STORE their first gradient writes: skip the step's zero fill of
    # the gradient bucket (the next backward overwrites it; engine.py "Deferred zeroing")
    defer_zero_grad: bool = True
    # pin the engine's host thread to one CPU (accelerator.pin_host_thread): a host-bound graphed step
    # then keeps its rate from process to process (profiles/r6_engine_graph_variance.txt).  Opt-in:
    # threads / processes the pinned thread starts later inherit the CPU.  DGT_PIN_HOST_THREAD=1 too
    pin_host_thread: bool = False


@dataclass
class DSConfig:
    train_batch_size: int
    train_micro_batch_size_per_gpu: int
    gradient_accumulation_steps: int
    world_size: int
    fp16_enabled: bool = False
    bf16_enabled: bool = False
    loss_scale: float = 0.0          # 0 = dynamic (fp16 only)
    initial_scale_power: int = 16
    gradient_clipping: float = 0.0
    steps_per_print: int = 10
    wall_clock_breakdown: bool = False
    prescale_gradients: bool = False
    gradient_predivide_factor: float = 1.0
    communication_data_type: Optional[str] = None
    zero: ZeroConfig = field(default_factory=ZeroConfig)
    optimizer: Optional[OptimizerConfig] = None
    scheduler: SchedulerConfig = field(default_factory=SchedulerConfig)
    amd: AMDConfig = field(default_factory=AMDConfig)
    raw: Dict[str, Any] = field(default_factory=dict)

    @property
    def zero_stage(self) -> int:
        return self.zero.stage

    @property
    def compute_dtype(self) -> str:
        if self.bf16_enabled:
            return "bf16"
        if self.fp16_enabled:
            return "fp16"
        return "fp32"

    def to_dict(self) -> Dict[str, Any]:
        return copy.deepcopy(self.raw)


def load_config_source(config: Union[str, os.PathLike, Dict[str, Any], None]) -> Dict[str, Any]:
    if config is None:
        return copy.deepcopy(REFERENCE_DS_CONFIG)
    if isinstance(config, dict):
        return copy.deepcopy(config)
    with open(config, "r") as fh:
        return json.load(fh)


def resolve_batch(tb: Optional[int], mb: Optional[int], gas: Optional[int], ws: int):
    """DeepSpeed's batch-parameter derivation (``_set_batch_related_parameters``)."""
    if tb is not None and mb is not None and gas is not None:
        pass
    elif tb is not None and mb is not None:
        gas = tb // mb // ws
    elif tb is not None and gas is not None:
        mb = tb // ws // gas
    elif mb is not None and gas is not None:
        tb = mb * gas * ws
    elif tb is not None:
        gas = 1
        mb = tb // ws
    elif mb is not None:
        gas = 1
        tb = mb * ws
    else:
        raise ConfigError("either train_batch_size or train_micro_batch_size_per_gpu must be set")
    if tb is None or tb <= 0 or mb is None or mb <= 0 or gas is None or gas <= 0:
        raise ConfigError(
            f"batch parameters must be positive: train_batch_size={tb} "
            f"micro_batch_per_gpu={mb} gradient_accumulation_steps={gas} (world_size={ws}); "
            f"train_batch_size must be divisible by world_size * gradient_accumulation_steps")
    if tb != mb * gas * ws:
        raise ConfigError(
            "Check batch related parameters. train_batch_size is not equal to "
            f"micro_batch_per_gpu * gradient_acc_step * world_size {tb} != {mb} * {gas} * {ws} "
            f"(train_batch_size={tb} is not divisible by world_size={ws}; pick a world size that "
            f"divides it or set train_micro_batch_size_per_gpu explicitly)")
    return tb, mb, gas


def parse_config(config: Union[str, os.PathLike, Dict[str, Any], None], world_size: int = 1) -> DSConfig:
    raw = load_config_source(config)
    tb, mb, gas = resolve_batch(raw.get("train_batch_size"), raw.get("train_micro_batch_size_per_gpu"),
                                raw.get("gradient_accumulation_steps"), world_size)

    fp16 = raw.get("fp16", {}) or {}
    bf16 = raw.get("bf16", raw.get("bfloat16", {})) or {}
    if fp16.get("enabled", False) and bf16.get("enabled", False):
        raise ConfigError("fp16 and bf16 cannot both be enabled")

    z = raw.get("zero_optimization", {}) or {}
    stage = int(z.get("stage", 0))
    if stage not in (0, 1, 2):
        raise ConfigError(f"zero_optimization.stage={stage} is not supported (0, 1 and 2 are)")
    zero = ZeroConfig(
        stage=stage,
        reduce_bucket_size=int(z.get("reduce_bucket_size", DEFAULT_BUCKET_BYTES // 4)),
        allgather_bucket_size=int(z.get("allgather_bucket_size", DEFAULT_BUCKET_BYTES // 4)),
        overlap_comm=bool(z.get("overlap_comm", True)),
        contiguous_gradients=bool(z.get("contiguous_gradients", True)),
        reduce_scatter=bool(z.get("reduce_scatter", True)),
    )

    opt = None
    if "optimizer" in raw:
        o = raw["optimizer"]
        p = o.get("params", {})
        t = str(o.get("type", "Adam"))
        if t.lower() not in ("adam", "adamw", "fusedadam"):
            raise ConfigError(f"optimizer type {t!r} not supported (Adam / AdamW)")
        opt = OptimizerConfig(type=t, lr=float(p.get("lr", 1e-3)),
                              betas=tuple(p.get("betas", (0.9, 0.999))),
                              eps=float(p.get("eps", 1e-8)),
                              weight_decay=float(p.get("weight_decay", 0.0)),
                              adamw=(t.lower() == "adamw") or bool(p.get("adam_w_mode", False)))

    sch = raw.get("scheduler", {}) or {}
    scheduler = SchedulerConfig(type=sch.get("type"), params=dict(sch.get("params", {})))
    if scheduler.type not in (None, "WarmupLR", "WarmupDecayLR"):
        raise ConfigError(f"scheduler {scheduler.type!r} not supported (WarmupLR / WarmupDecayLR)")

    a = raw.get("amd", {}) or {}
    amd = AMDConfig(allreduce=str(a.get("allreduce", "auto")),
                    oneshot_max_bytes=int(a.get("oneshot_max_bytes", 256 * 1024)),
                    hip_graph=bool(a.get("hip_graph", False)),
                    debug_sync_streams=bool(a.get("debug_sync_streams", False)),
                    fused_linear=None if a.get("fused_linear") is None else bool(a["fused_linear"]),
                    graph_module=bool(a.get("graph_module", False)),
                    graph_tail=bool(a.get("graph_tail", True)),
                    graph_bind_inputs=bool(a.get("graph_bind_inputs", True)),
                    direct_backward=bool(a.get("direct_backward", True)),
                    defer_zero_grad=bool(a.get("defer_zero_grad", True)),
                    pin_host_thread=bool(a.get("pin_host_thread", False)))
    if amd.allreduce not in ("auto", "rccl", "oneshot"):
        raise ConfigError(f"amd.allreduce={amd.allreduce!r}: expected auto|rccl|oneshot")

    return DSConfig(
        train_batch_size=tb, train_micro_batch_size_per_gpu=mb, gradient_accumulation_steps=gas,
        world_size=world_size,
        fp16_enabled=bool(fp16.get("enabled", False)),
        bf16_enabled=bool(bf16.get("enabled", False)),
        loss_scale=float(fp16.get("loss_scale", 0.0)),
        initial_scale_power=int(fp16.get("initial_scale_power", 16)),
        gradient_clipping=float(raw.get("gradient_clipping", 0.0)),
        steps_per_print=int(raw.get("steps_per_print", 10)),
        wall_clock_breakdown=bool(raw.get("wall_clock_breakdown", False)),
        prescale_gradients=bool(raw.get("prescale_gradients", False)),
        gradient_predivide_factor=float(raw.get("gradient_predivide_factor", 1.0)),
        communication_data_type=raw.get("communication_data_type"),
        zero=zero, optimizer=opt, scheduler=scheduler, amd=amd, raw=raw,
    )
