"""Device-resident trainer for the reference model (the fused HIP path of ``train.py``).

The reference's hot loop (``train.py:99-117``) does, per step: DataLoader collate on the CPU, two
H2D copies, ~30 ATen/cuBLAS launches, a DeepSpeed flatten -> NCCL all-reduce -> unflatten, seven
foreach-Adam launches and a blocking ``loss.item()``.  This trainer keeps the whole problem on the
GPU instead:

* dataset, parameters and Adam moments live in HBM for the whole run; the sampler's per-epoch
  index plan (bit-exact ``DistributedSampler``) is uploaded once per epoch;
* ``impl="fused"``: ONE kernel launch per epoch runs every step (``csrc/tiny_mlp.hip``),
  exchanging gradients with the peers through the IPC mailboxes over xGMI when world_size > 1;
* ``impl="graph"``: per step a fused fwd+bwd kernel -> native RCCL all-reduce -> fused flat Adam
  with a device-resident step counter, one epoch of steps captured in a HIP graph and replayed
  (the multi-GPU path when IPC mailboxes are unavailable);
* ``impl="stepwise"``: the same kernels launched eagerly with ProcessGroupNCCL (RCCL) in between
  (the A/B baseline for the fused kernel);
* ``impl="torch"``: the same math in plain PyTorch (CPU / gloo, and the numerics reference).

The epoch's mean loss is accumulated on the device and read once per epoch, giving the same
printed value as the reference's per-step ``loss.item()`` sum.

Exchange robustness (the fused path at world size > 1): before training, the mailboxes pass the
one-shot all-reduce self-test, then the in-kernel exchange's line format is chosen by a stress
test of >= 1000 exchanges whose payloads expose any torn or lost line (``DGT_XCH_LINE``: LL3,
16-byte lines, if it passes, else LL2, 8-byte atomic pairs, else RCCL), then 8 training steps are
checked against the RCCL path.  At run time every epoch starts from a snapshot (params, moments,
step counters); a kernel-reported exchange timeout or a replica divergence at the epoch's end
makes every rank restore it and re-run the epoch on the RCCL path (``exchange_fallback``, logged
to stderr, ``DGT_METRICS_JSONL`` and ``DGT_HEALTH_LOG``), unless ``strict_exchange`` keeps it
fatal.

``zero_stage=1`` (DeepSpeed ZeRO-1): the fused kernel's exchange becomes reduce-scatter
of the gradients to lane owners, the owner's Adam on the moments only it keeps, and all-gather of
the updated parameters; checkpoints hold one ``zero_pp_rank_{r}`` shard of owned elements per rank.
"""
from __future__ import annotations

import functools
import os
import sys
from typing import Any, Dict, List, Optional

import torch

from .. import data as dgt_data
from ..accelerator import get_accelerator
from ..models.simple_net import SimpleNet, pack_simple_net, simple_net_layout, simple_net_numel
from ..ops import _ext
from ..ops.adam import adam_flat_
from ..ops.reference import adam_flat_reference_, tiny_mlp_step_reference
from ..parallel import comm
from . import checkpoint as ckpt
from ..utils import tracing
from ..utils.fault import FaultInjector
from ..utils.metrics import MetricsSink, health_event
from .optim_state import adam_state_to_flat, flat_to_adam_state

IMPLS = ("auto", "fused", "graph", "stepwise", "torch")
LINES = {"ll3": 3, "ll2": 2}


def _raw_stream(index: int) -> int:
    return torch._C._cuda_getCurrentRawStream(index)


def line_candidates() -> List[int]:
    """Exchange line formats to try, in order (``DGT_XCH_LINE=auto|ll3|ll2``): auto = LL3 (three
    payload floats per 16-byte line, fewest instructions) if its stress test passes, else LL2
    (two 8-byte {payload, tag} pairs per line: needs only 64-bit single-copy atomicity)."""
    mode = os.environ.get("DGT_XCH_LINE", "auto")
    if mode == "auto":
        return [3, 2]
    if mode not in LINES:
        raise ValueError(f"DGT_XCH_LINE must be auto, ll3 or ll2, got {mode!r}")
    return [LINES[mode]]


def stress_steps() -> int:
    return max(1, int(os.environ.get("DGT_XCH_STRESS_STEPS", "2000")))


def zero1_owner_map(n_features: int, hidden: int, world_size: int) -> torch.Tensor:
    """Owning rank of every flat parameter under the fused kernel's ZeRO-1 exchange: the kernel
    keeps W1[j][k] / b1[j] in lane (j % 16, slot) of wave j // 16 and W2 in lanes 0-3 of each DPP
    row (``csrc/tiny_mlp.hip`` TinyCfg::slot_index / bw_index); lane l is owned by rank l % world;
    b2 is replicated; each rank writes its state back from a lane it owns (lane = rank), so every
    rank's copy is current and rank 0's stands for the shard."""
    F, H = n_features, hidden
    nkt = (F + 1 + 15) // 16
    rem = F + 1 - 16 * (nkt - 1)
    nsl = 4 * (nkt - 1) + (rem + 3) // 4
    g_b1, g_w2, g_b2 = H * F, H * F + H, H * F + 2 * H
    owner = torch.full((simple_net_numel(F, H),), -1, dtype=torch.int64)
    for w in range(H // 16):
        for l in range(64):
            lr, lq, own = l & 15, l >> 4, l % world_size
            for i in range(nsl):
                k = 16 * (i >> 2) + lq + 4 * (i & 3)
                if k < F:
                    owner[(16 * w + lr) * F + k] = own
                elif k == F:
                    owner[g_b1 + 16 * w + lr] = own
            if lr < 4:
                owner[g_w2 + 16 * w + 4 * lq + lr] = own
    owner[g_b2] = 0
    assert bool((owner >= 0).all()), "every parameter has an owner lane"
    return owner


class ReplicaDivergence(RuntimeError):
    """Data-parallel replicas ended an epoch with different parameters (a corrupted exchange)."""


XSUM_WORDS = 2048  # 2 per thread of the fused kernel (<= 1024 threads); unused threads stay 0


def zero1_checksum_mismatch(per_rank: List[torch.Tensor], world_size: int) -> Optional[str]:
    """Check the ZeRO-1 kernel's transfer checksums (csrc/dgt_common.h Exchange::xsum) of every rank.
    Thread t's lane l = t % 64 is owned by rank l % world_size.  Word 2t: the owner's XOR of the
    parameters it all-gathered must equal every other rank's XOR of what it received.  Word 2t + 1:
    the owner's XOR of the gradients it received must equal the XOR over the other ranks of what
    they sent.  Returns a description of the first mismatch, or None."""
    xs = torch.stack([t.view(-1, 2).to(torch.int64) for t in per_rank])  # [ranks, threads, 2]
    n = xs.shape[1]
    owner = (torch.arange(n) % 64) % world_size
    ag = xs[:, :, 0]
    bad_ag = (ag != ag.gather(0, owner.view(1, -1)).expand_as(ag)).any(0)
    acc = torch.zeros(n, dtype=torch.int64)
    for p in range(world_size):  # XOR over every rank: the owner's received word cancels the senders'
        acc ^= xs[p, :, 1]
    bad_rs = acc != 0
    if bool(bad_ag.any()):
        t = int(torch.nonzero(bad_ag)[0])
        o = int(owner[t])
        r = int(torch.nonzero(ag[:, t] != ag[o, t])[0])
        return f"parameters all-gathered by rank {o} arrived altered on rank {r} (thread {t})"
    if bool(bad_rs.any()):
        t = int(torch.nonzero(bad_rs)[0])
        return f"gradients reduce-scattered to rank {int(owner[t])} arrived altered (thread {t})"
    return None


class ExchangeFailure(RuntimeError):
    """The fused kernel's in-kernel exchange failed on some rank (timeout or replica divergence)."""


def fused_supported(n_features: int, hidden: int, batch_size: int) -> bool:
    if not (get_accelerator().name == "hip" and _ext.available()):
        return False
    return bool(_ext.require().tiny_mlp_supported(n_features, hidden)) and batch_size <= 16


class TinyMLPTrainer:
    def __init__(self, model: SimpleNet, x: torch.Tensor, y: torch.Tensor, batch_size: int = 4,
                 lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 adamw: bool = False, device: Optional[torch.device] = None, impl: str = "auto",
                 sampler_seed: int = 0, ds_config: Optional[Dict[str, Any]] = None, use_ipc: bool = True,
                 exchange_timeout_s: Optional[float] = None, zero_stage: int = 0,
                 strict_exchange: Optional[bool] = None):
        if impl not in IMPLS:
            raise ValueError(f"impl must be one of {IMPLS}")
        if zero_stage not in (0, 1):
            raise ValueError("TinyMLPTrainer supports zero_stage 0 or 1")
        self.F = model.n_features
        self.H = model.hidden
        self.B = batch_size
        self.device = device or get_accelerator().device()
        self.rank = comm.get_rank()
        self.world_size = comm.get_world_size()
        self.lr, self.betas, self.eps = float(lr), (float(betas[0]), float(betas[1])), float(eps)
        self.weight_decay, self.adamw = float(weight_decay), bool(adamw)
        self.sampler_seed = sampler_seed
        self.ds_config = ds_config or {}
        self.global_steps = 0
        self.global_samples = 0
        self.channel = None
        self.zero_stage = zero_stage
        self.line = 3            # exchange line format of the fused kernel (set by the stress test)
        self.xch_report: List[Dict[str, Any]] = []  # start-up self-tests of the exchange
        self.fallbacks: List[Dict[str, Any]] = []   # run-time exchange fallbacks
        self.strict_exchange = (os.environ.get("DGT_STRICT_EXCHANGE", "0") not in ("", "0")
                                if strict_exchange is None else bool(strict_exchange))
        self._corrupt_off = False  # the torch path's corrupt fault is one-shot (a re-run is clean)

        if impl == "auto":
            impl = "fused" if (self.device.type == "cuda" and fused_supported(self.F, self.H, self.B)) else (
                "torch" if self.device.type == "cpu" else "stepwise")
        if impl in ("fused", "stepwise", "graph"):
            if self.device.type != "cuda":
                raise RuntimeError(f"impl={impl!r} needs a GPU")
            if not fused_supported(self.F, self.H, self.B):
                raise RuntimeError(f"no fused kernel for F={self.F} H={self.H} B={self.B}")
        self.impl = impl

        self.numel = simple_net_numel(self.F, self.H)
        self.padded = (self.numel + 3) // 4 * 4
        self.segments = [(off, shp) for _, shp, off in simple_net_layout(self.F, self.H)]
        flat = torch.zeros(self.padded, dtype=torch.float32)
        flat[: self.numel] = pack_simple_net(model)
        self.params = flat.to(self.device)
        comm.broadcast_(self.params, 0)  # DeepSpeed broadcasts the model at initialize
        self.exp_avg = torch.zeros_like(self.params)
        self.exp_avg_sq = torch.zeros_like(self.params)
        self.grad = torch.zeros_like(self.params)
        self.model = model
        self.x = x.to(self.device, torch.float32).contiguous()
        self.y = y.to(self.device, torch.float32).reshape(-1).contiguous()
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=self.device)
        self.status = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.exchange_timeout_s = float(exchange_timeout_s if exchange_timeout_s is not None
                                        else os.environ.get("DGT_EXCHANGE_TIMEOUT_S", 60.0))
        self.faults = FaultInjector.from_env(self.rank)
        self.metrics = MetricsSink.from_env(self.rank)

        # ZeRO-1 exchange inside the fused kernel (one rank: nothing to shard, the plain kernel)
        self.zero1 = self.zero_stage == 1 and self.world_size > 1
        self._auto_fallback = False
        if self.impl == "fused" and self.world_size > 1:
            self.channel = self._open_channel() if use_ipc else None
            if self.channel is None:
                self.impl = "graph" if comm.backend_name() == "nccl" else "stepwise"
                self._auto_fallback = True
        self._graph = None
        self.rccl = None
        self._lh = None  # lean fused launcher (created on the first fused launch)
        self._lh_stream = None
        self._ws = None  # the fused kernel's bias-correction workspace (it fills it itself)
        self._xsum = None  # ZeRO-1 transfer checksums (zero1_checksum_mismatch)
        if self.impl == "fused":
            self.reserve(self.steps_per_epoch())
        if self.impl == "graph":
            try:
                self._setup_graph()
            except Exception as e:
                # an automatic fallback must not take the job down: every rank agrees on the
                # plain ProcessGroupNCCL path instead
                if not self._auto_fallback:
                    raise
                print(f"[dgt] graph path unavailable ({e}); using stepwise", flush=True)
                self.impl = "stepwise"
        if self._auto_fallback and self.world_size > 1:
            agreed = comm.all_reduce_max(1.0 if self.impl == "stepwise" else 0.0)
            if agreed > 0 and self.impl != "stepwise":
                self.close_graph_resources()
                self.impl = "stepwise"
        if self.impl != "fused":
            # the RCCL / PyTorch paths run ZeRO-1 with ZeRO-0 math (replicated moments: 1409 params
            # make the shard's memory saving moot); checkpoints are still written as ZeRO-1 shards
            self.zero1 = False

    # ------------------------------------------------------------------ setup helpers
    def _open_channel(self):
        from ..parallel.ipc import IpcChannel, ipc_disabled_by_env
        if ipc_disabled_by_env() or self.world_size > 8:
            return None
        try:
            need = int(_ext.require().tiny_mlp_exchange_floats(self.F, self.H))
            ch = IpcChannel(max(need, self.padded), self.device, timeout_s=self.exchange_timeout_s)
        except Exception:
            return None
        if not ch.selftest():
            ch.close()
            return None
        line = self._pick_line(ch)
        if line is None or not self._exchange_selftest(ch):
            ch.close()
            return None
        return ch

    def _pick_line(self, ch) -> Optional[int]:
        """The first line format (``line_candidates``) whose stress test passes on every rank."""
        for line in line_candidates():
            ok, detail = self._stress(ch, line, stress_steps())
            self.xch_report.append({"test": "stress", "line": f"ll{line}", "ok": ok, **detail})
            if ok:
                self.line = line
                return line
            if self.rank == 0:
                print(f"[dgt] exchange stress test failed for LL{line} ({detail}); "
                      f"{'trying the next line format' if line != line_candidates()[-1] else 'using RCCL'}",
                      file=sys.stderr, flush=True)
        return None

    def _stress(self, ch, line: int, n_steps: int, timeout_s: float = 10.0):
        """``n_steps`` exchanges of the fused kernel's own mailbox layout and line format with
        payloads that expose any torn line (``tiny_xch_stress``); every rank agrees on the verdict."""
        ops = _ext.require()
        status = torch.zeros(1, dtype=torch.int32, device=self.device)
        errors = torch.zeros(1, dtype=torch.int32, device=self.device)
        err, st = 0, 0
        try:
            ops.tiny_xch_stress(self.F, self.H, ch.data_ptrs, self.rank, self.world_size, ch.stride,
                                ch.next_seq(n_steps), int(timeout_s * 100_000_000), line, n_steps, status, errors)
            torch.cuda.synchronize(self.device)
            err, st = int(errors.item()), int(status.item())
        except Exception as e:
            print(f"[dgt] exchange stress test raised: {e}", file=sys.stderr, flush=True)
            st = -1
        bad_words = comm.all_reduce_max(float(err))
        worst = comm.all_reduce_max(float(st != 0))
        ok = bad_words == 0 and worst == 0
        return ok, {"steps": n_steps, "max_bad_words": int(bad_words), "timeout_or_error": bool(worst)}

    def _exchange_selftest(self, ch, n_steps: int = 8, timeout_s: float = 10.0) -> bool:
        """Drive the training kernel's OWN in-kernel exchange (not the stand-alone one-shot
        all-reduce of ``IpcChannel.selftest``) for ``n_steps`` steps of this rank's first batches on
        scratch copies of the state, then check (a) the kernel reported no timeout, (b) the result
        matches the RCCL path (per-step gradient -> process-group all-reduce -> exact flat Adam)
        within fp32 tolerance, and (c) every rank holds bit-identical parameters.  Every rank
        issues the same collectives whatever happens, and all ranks agree on the verdict."""
        ops = _ext.require()
        plan, counts = self.epoch_plan(1)
        plan, counts = plan[:n_steps].contiguous(), counts[:n_steps].contiguous()
        n = int(plan.shape[0])
        p = self.params.clone()
        m, v = torch.zeros_like(p), torch.zeros_like(p)
        loss = torch.zeros(1, dtype=torch.float64, device=self.device)
        status = torch.zeros(1, dtype=torch.int32, device=self.device)
        ok = True
        try:
            ops.tiny_mlp_train(self.x, self.y, plan, counts, p, m, v, loss, status, self.F, self.H, self.lr,
                               self.betas[0], self.betas[1], self.eps, self.weight_decay, self.adamw, 0,
                               ch.data_ptrs, self.rank, self.world_size, ch.stride, ch.next_seq(n),
                               int(timeout_s * 100_000_000), -1, None, int(self.zero1), self.line)
            torch.cuda.synchronize(self.device)
            ok = int(status.item()) == 0
        except Exception as e:
            print(f"[dgt] in-kernel exchange self-test raised: {e}", flush=True)
            ok = False
        rp = self.params.clone()
        rm, rv, g = torch.zeros_like(rp), torch.zeros_like(rp), torch.zeros_like(rp)
        lacc = torch.zeros(1, dtype=torch.float64, device=self.device)
        for s in range(n):  # unconditional: every rank issues the same collectives
            ops.tiny_mlp_grad(self.x, self.y, plan, counts, s, rp, g, lacc, self.F, self.H)
            comm.all_reduce_(g)
            adam_flat_(rp, g, rm, rv, s + 1, self.lr, self.betas[0], self.betas[1], self.eps, self.weight_decay,
                       self.adamw, grad_scale=1.0 / self.world_size)
        ok = ok and bool(torch.allclose(p, rp, rtol=1e-4, atol=1e-6))
        ref = p.clone()
        comm.broadcast_(ref, 0)
        ok = ok and bool(torch.equal(p, ref))
        agreed = comm.all_reduce_max(0.0 if ok else 1.0) == 0.0
        self.xch_report.append({"test": "train_steps", "line": f"ll{self.line}", "ok": agreed, "steps": n})
        return agreed

    def _setup_graph(self) -> None:
        if comm.collectives_on(self.world_size):
            if comm.backend_name() != "nccl":
                raise RuntimeError("impl='graph' needs RCCL (one GPU per rank)")
            from ..parallel.rccl import RcclComm
            self.rccl = RcclComm(self.device)
        self.step_dev = torch.zeros((), dtype=torch.int64, device=self.device)
        self.step_ticket = torch.zeros((), dtype=torch.int32, device=self.device)  # Adam advances step_dev
        self._gsteps = self.steps_per_epoch()
        self._gplan = torch.full((self._gsteps, self.B), -1, dtype=torch.int32, device=self.device)
        self._gcounts = torch.ones(self._gsteps, dtype=torch.int32, device=self.device)

    def _graph_step(self, plan, counts, s: int) -> None:
        ops = _ext.require()
        ops.tiny_mlp_grad(self.x, self.y, plan, counts, s, self.params, self.grad, self.loss_acc, self.F, self.H)
        if self.rccl is not None:
            self.rccl.all_reduce(self.grad)
        adam_flat_(self.params, self.grad, self.exp_avg, self.exp_avg_sq, 1, self.lr, self.betas[0], self.betas[1],
                   self.eps, self.weight_decay, self.adamw, grad_scale=1.0 / self.world_size, step_dev=self.step_dev,
                   step_ticket=self.step_ticket)

    def _capture(self) -> None:
        # warm the kernels once outside capture, then restore the state they touched
        saved = [t.clone() for t in (self.params, self.exp_avg, self.exp_avg_sq, self.loss_acc, self.step_dev)]
        self._graph_step(self._gplan, self._gcounts, 0)
        torch.cuda.synchronize(self.device)
        for t, v in zip((self.params, self.exp_avg, self.exp_avg_sq, self.loss_acc, self.step_dev), saved):
            t.copy_(v)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for s in range(self._gsteps):
                self._graph_step(self._gplan, self._gcounts, s)
        self._graph = g

    @property
    def exchange(self) -> str:
        if self.world_size == 1:
            return "none"
        if self.impl == "fused":
            return f"ipc-{'zero1' if self.zero1 else 'oneshot'}-xgmi/ll{self.line}"
        if self.impl == "graph":
            return "rccl-native-in-hipgraph"
        return f"{comm.backend_name()}-allreduce"

    def steps_per_epoch(self) -> int:
        return dgt_data.steps_per_epoch(self.x.shape[0], self.world_size, self.B)

    def epoch_plan(self, epoch: int):
        idx = dgt_data.shard_indices(self.x.shape[0], self.world_size, self.rank, epoch, self.sampler_seed)
        plan = dgt_data.batch_plan(idx, self.B)
        counts = (plan >= 0).sum(1).to(torch.int32)
        return plan.to(self.device), counts.to(self.device)

    # ------------------------------------------------------------------ training
    def run_plan(self, plan: torch.Tensor, counts: torch.Tensor) -> None:
        """Run len(plan) optimizer steps (asynchronously on GPU); loss accumulates into loss_acc."""
        n = int(plan.shape[0])
        if n == 0:
            return
        if self.impl == "fused" and self._lean_ok(plan, counts, n):
            # Adam's bias corrections of steps global_steps+1 .. +n are formed inside the kernel
            ch = self.channel
            seq = ch.next_seq(n) if ch is not None else 0
            stream = _raw_stream(self.device.index)
            if stream != self._lh_stream:
                self._clib.dgt_tiny_launcher_set_stream(self._lh, stream)
                self._lh_stream = stream
            self.reserve(n)
            rc = self._clib.dgt_tiny_launch(self._lh, plan.data_ptr(), counts.data_ptr(), n, plan.shape[1],
                                            self.global_steps, seq, self._ws_ptr)
            if rc != 0:
                raise RuntimeError(f"dgt: fused training kernel launch failed (hipError {rc})")
            self.global_steps += n
        elif self.impl == "fused":  # the validating op path (it raises on a malformed plan)
            ops = _ext.require()
            ch = self.channel
            seq = ch.next_seq(n) if ch is not None else 0
            ops.tiny_mlp_train(self.x, self.y, plan, counts, self.params, self.exp_avg, self.exp_avg_sq,
                               self.loss_acc, self.status, self.F, self.H, self.lr, self.betas[0], self.betas[1],
                               self.eps, self.weight_decay, self.adamw, self.global_steps,
                               ch.data_ptrs if ch else [], self.rank,
                               self.world_size, ch.stride if ch else 0, seq,
                               ch.timeout_ticks if ch else 0, self.faults.corrupt_step(), self._ws,
                               int(self.zero1), self.line, self._xsum_ptr())
            self.global_steps += n
        elif self.impl == "graph":
            self.step_dev.fill_(self.global_steps)
            s = 0
            while n - s >= self._gsteps:
                if self._graph is None:
                    self._capture()
                self._gplan.copy_(plan[s:s + self._gsteps])
                self._gcounts.copy_(counts[s:s + self._gsteps])
                self._graph.replay()
                s += self._gsteps
            for r in range(s, n):  # tail shorter than one captured epoch: eager launches
                self._graph_step(plan, counts, r)
            self.global_steps += n
        elif self.impl == "stepwise":
            ops = _ext.require()
            for s in range(n):
                ops.tiny_mlp_grad(self.x, self.y, plan, counts, s, self.params, self.grad, self.loss_acc,
                                  self.F, self.H)
                comm.all_reduce_(self.grad)  # no-op at world size 1 unless DGT_FORCE_COLLECTIVES
                self.global_steps += 1
                adam_flat_(self.params, self.grad, self.exp_avg, self.exp_avg_sq, self.global_steps, self.lr,
                           self.betas[0], self.betas[1], self.eps, self.weight_decay, self.adamw,
                           grad_scale=1.0 / self.world_size)
        else:
            plan_c, counts_c = plan.cpu(), counts.cpu()
            for s in range(n):
                rows = plan_c[s, : int(counts_c[s])].long().to(self.device)
                loss, g = tiny_mlp_step_reference(self.params, self.x[rows], self.y[rows], self.F, self.H,
                                                  grad_out=self.grad)
                self.loss_acc += loss
                comm.all_reduce_(self.grad)
                self.global_steps += 1
                self._maybe_corrupt_torch()
                adam_flat_reference_(self.params, self.grad, self.exp_avg, self.exp_avg_sq, self.global_steps,
                                     self.lr, self.betas[0], self.betas[1], self.eps, self.weight_decay,
                                     self.adamw, grad_scale=1.0 / self.world_size)
        self.global_samples += n * self.B * self.world_size
        self.faults.maybe_fire(self.global_steps)

    def bind_launch(self, plan: torch.Tensor, counts: torch.Tensor, prepared: bool = True):
        """``run_plan(plan, counts)`` as a zero-argument callable whose per-call host work is one
        ctypes call and the step bookkeeping: the plan checks, the stream lookup, the workspace
        sizing, the argument block and (``prepared``) the kernel lookup happen here, once, and the
        launch passes the whole argument block as one buffer (``dgt_tiny_launch_prepared`` ->
        hipModuleLaunchKernel); ``prepared=False`` keeps the per-launch entry point
        (``dgt_tiny_launch`` -> hipLaunchKernel).  Valid while the current stream stays the one
        bound here.  Paths other than the dispatcher-free fused launch get ``run_plan`` itself."""
        n = int(plan.shape[0])
        if not (self.impl == "fused" and n and self._lean_ok(plan, counts, n)):
            return functools.partial(self.run_plan, plan, counts)
        self.reserve(n)
        stream = _raw_stream(self.device.index)
        if stream != self._lh_stream:
            self._clib.dgt_tiny_launcher_set_stream(self._lh, stream)
            self._lh_stream = stream
        ch = self.channel
        pp, cp, bmax, ws = plan.data_ptr(), counts.data_ptr(), int(plan.shape[1]), self._ws_ptr
        if prepared:
            import ctypes
            import weakref
            err = ctypes.c_int(0)
            handle = self._clib.dgt_tiny_prepare(self._lh, pp, cp, n, bmax, ws, ctypes.byref(err))
            if not handle:
                raise RuntimeError(f"dgt: preparing the fused training kernel launch failed (hipError {err.value})")
            fn = self._clib.dgt_tiny_launch_prepared
            keep = (plan, counts, self._ws)  # the prepared block holds their device addresses

            def launch() -> None:
                seq = ch.next_seq(n) if ch is not None else 0
                rc = fn(handle, self.global_steps, seq)
                if rc != 0:
                    raise RuntimeError(f"dgt: fused training kernel launch failed (hipError {rc})")
                self.global_steps += n
            launch.keep = keep
            weakref.finalize(launch, self._clib.dgt_tiny_prepared_free, handle)
            return launch
        fn, lh = self._clib.dgt_tiny_launch, self._lh

        def launch() -> None:
            seq = ch.next_seq(n) if ch is not None else 0
            rc = fn(lh, pp, cp, n, bmax, self.global_steps, seq, ws)
            if rc != 0:
                raise RuntimeError(f"dgt: fused training kernel launch failed (hipError {rc})")
            self.global_steps += n
        return launch

    def reserve(self, n_steps: int) -> None:
        """Size the fused kernel's workspace for launches of up to ``n_steps`` steps (the kernel fills
        it with its own steps' Adam bias corrections; this is allocation only, no per-step work)."""
        need = (max(int(n_steps), 1) + 1) * 2
        if self.impl == "fused" and (self._ws is None or self._ws.numel() < need):
            self._ws = torch.empty(need, dtype=torch.float32, device=self.device)
            self._ws_ptr = self._ws.data_ptr()

    def _lean_ok(self, plan: torch.Tensor, counts: torch.Tensor, n: int) -> bool:
        """Whether this launch can take the dispatcher-free path: a well-formed device plan (the
        launcher itself was validated once, at creation)."""
        if not (plan.is_cuda and plan.dtype == torch.int32 and plan.dim() == 2 and plan.is_contiguous()
                and counts.is_cuda and counts.dtype == torch.int32 and counts.is_contiguous()
                and counts.numel() == n and 1 <= plan.shape[1] <= 16):
            return False
        if self._lh is None:
            ch = self.channel
            self._lh = int(_ext.require().tiny_launcher_create(
                self.x, self.y, self.params, self.exp_avg, self.exp_avg_sq, self.loss_acc, self.status, self.F,
                self.H, self.lr, self.betas[0], self.betas[1], self.eps, self.weight_decay, self.adamw,
                ch.data_ptrs if ch else [], self.rank, self.world_size, ch.stride if ch else 0,
                ch.timeout_ticks if ch else 0, self.faults.corrupt_step(), int(self.zero1), self.line,
                self._xsum_ptr()))
            self._lh_stream = _raw_stream(self.device.index)  # the launcher was bound to it
            self._clib = _ext.c_lib()
        return True

    def _drop_launcher(self) -> None:
        if getattr(self, "_lh", None):
            try:
                _ext.require().tiny_launcher_destroy(self._lh)
            except Exception:
                pass
        self._lh = None

    def check(self) -> None:
        """Raise if a kernel reported a failure (cross-GPU timeout, bad shape)."""
        if self.device.type == "cuda":
            st = int(self.status.item())
            if st == 0 and self.channel is not None:
                st = self.channel.check_status()
            if st != 0:
                raise RuntimeError(f"fused training kernel failed with status {st} "
                                   f"({'cross-GPU exchange timeout' if st == 1 else 'bad launch shape'})")

    def device_barrier(self) -> bool:
        """Queue a device-side barrier over this trainer's IPC mailboxes on the current stream
        (``IpcChannel.barrier``); False when there is none (1 rank, or the exchange fell back to
        RCCL), so the caller uses the process group's barrier.  Failures surface in ``check()``."""
        ch = self.channel
        if ch is None or not ch.healthy or self.world_size == 1:
            return False
        ch.barrier()
        return True

    def verify_replicas(self) -> None:
        """Raise ReplicaDivergence on EVERY rank unless all ranks hold bit-identical parameters
        (data-parallel training keeps them identical; only a corrupted exchange breaks that) and,
        on the ZeRO-1 kernel, every transfer arrived as sent (a corrupted parameter all-gather is
        overwritten by the next step's, so identical replicas alone do not prove a clean epoch)."""
        if self.world_size == 1:
            return
        ref = self.params.clone()
        comm.broadcast_(ref, 0)
        bad = comm.all_reduce_max(0.0 if bool(torch.equal(self.params, ref)) else 1.0)
        if bad > 0:
            raise ReplicaDivergence(f"data-parallel replicas diverged by optimizer step {self.global_steps} "
                                    f"(impl={self.impl}, exchange={self.exchange})")
        if self._xsum is not None and self.zero1 and self.impl == "fused":
            why = zero1_checksum_mismatch(comm.all_gather_object(self._xsum.cpu()), self.world_size)
            if why:
                raise ReplicaDivergence(f"ZeRO-1 exchange transfer corrupted by optimizer step {self.global_steps}: "
                                        f"{why} (exchange={self.exchange})")

    def _xsum_ptr(self) -> int:
        """Device address of the ZeRO-1 transfer checksums (0 = not on the ZeRO-1 kernel)."""
        if not (self.zero1 and self.impl == "fused" and self.device.type == "cuda"):
            return 0
        if self._xsum is None:
            self._xsum = torch.zeros(XSUM_WORDS, dtype=torch.int32, device=self.device)
        return self._xsum.data_ptr()

    def _torch_corrupt_spec(self):
        spec = self.faults.spec
        ok = (spec is not None and spec.mode == "corrupt" and spec.step is not None and spec.rank is not None
              and not self._corrupt_off)
        return spec if ok else None

    def _maybe_corrupt_torch(self) -> None:
        """The ``corrupt`` fault on the plain-PyTorch path (CPU rehearsal of the fused kernel's):
        rank RANK + 1 receives a gradient sum off by 1.0 in one element at step STEP, once."""
        spec = self._torch_corrupt_spec()
        if (spec is not None and self.world_size > 1 and self.global_steps == spec.step
                and self.rank == (spec.rank + 1) % self.world_size):
            self.grad[0] += 1.0

    def _snapshot(self):
        return ([t.clone() for t in (self.params, self.exp_avg, self.exp_avg_sq)],
                (self.global_steps, self.global_samples))

    def _restore(self, snap) -> None:
        (p, m, v), (steps, samples) = snap
        for dst, src in zip((self.params, self.exp_avg, self.exp_avg_sq), (p, m, v)):
            dst.copy_(src)
        self.global_steps, self.global_samples = steps, samples
        self.status.zero_()

    def _can_fall_back(self) -> bool:
        # the same answer on every rank (it decides whether the ranks re-run an epoch together)
        return self.world_size > 1 and not self.strict_exchange and (
            self.impl == "fused" or (self.impl == "torch" and self._torch_corrupt_spec() is not None))

    def _epoch_failure(self) -> Optional[str]:
        """Why this epoch's result cannot be trusted on SOME rank (agreed by every rank), or None."""
        local = None
        try:
            self.check()
        except RuntimeError as e:
            local = str(e)
        if self.world_size > 1 and comm.all_reduce_max(1.0 if local else 0.0) > 0:
            return local or "a peer's fused kernel reported an exchange failure"
        if local:
            return local
        try:
            self.verify_replicas()
        except ReplicaDivergence as e:
            return str(e)
        return None

    def run_epoch(self, epoch: int) -> float:
        plan, counts = self.epoch_plan(epoch)
        snap = self._snapshot() if self._can_fall_back() else None
        self.loss_acc.zero_()
        if self._xsum is not None:
            self._xsum.zero_()  # this epoch's transfers only
        with tracing.range(f"dgt.{self.impl}.epoch{epoch}"):  # the fused path: ONE kernel launch
            self.run_plan(plan, counts)
        with tracing.range("dgt.epoch_sync"):
            loss_sum = float(self.loss_acc.item())  # the epoch's single host sync
        with tracing.range("dgt.replica_check"):
            # one 5.6 KB broadcast per epoch: silent corruption is caught here
            why = self._epoch_failure() if self.world_size > 1 else None
            if why is None and self.world_size == 1:
                self.check()
        if why is not None:
            if snap is None:  # strict (or nothing to fall back to): the job fails loudly
                if "diverged" in why:
                    raise ReplicaDivergence(why)
                raise ExchangeFailure(why)
            return self._fall_back_and_rerun(epoch, snap, why)
        return loss_sum / max(1, int(plan.shape[0]))

    def _fall_back_and_rerun(self, epoch: int, snap, why: str) -> float:
        """Every rank restores the epoch-start snapshot, leaves the in-kernel exchange for the RCCL
        path (HIP-graph-captured native RCCL if every rank can set it up, else ProcessGroupNCCL /
        gloo step by step) and re-runs the epoch there; the job then continues on that path."""
        was = f"{self.impl}/{self.exchange}"
        self._restore(snap)
        if self.zero1:  # leaving the sharded kernel: every rank needs every element's moments
            self._gather_zero1_moments()
            self.zero1 = False
        if self.impl == "fused":
            self._drop_launcher()
            if self.channel is not None:
                self.channel.close()
                self.channel = None
            self.impl = "graph" if comm.backend_name() == "nccl" else "stepwise"
            if self.impl == "graph":
                try:
                    self._setup_graph()
                    ok = 0.0
                except Exception as e:
                    print(f"[dgt] graph path unavailable ({e})", file=sys.stderr, flush=True)
                    ok = 1.0
                if comm.all_reduce_max(ok) > 0:  # every rank takes the same path
                    self.close_graph_resources()
                    self.impl = "stepwise"
        self._corrupt_off = True
        rec = {"event": "exchange_fallback", "epoch": epoch, "from": was, "to": f"{self.impl}/{self.exchange}",
               "reason": why, "rank": self.rank, "world_size": self.world_size, "global_steps": self.global_steps}
        self.fallbacks.append(rec)
        print(f"[dgt] WARNING: exchange_fallback at epoch {epoch}: {why}; restored the epoch-start state and "
              f"re-running the epoch on {rec['to']}", file=sys.stderr, flush=True)
        self.metrics.log(rec)
        health_event(rec)
        return self.run_epoch(epoch)

    # ------------------------------------------------------------------ state
    def sync_model(self) -> SimpleNet:
        flat = self.params[: self.numel].detach().cpu()
        with torch.no_grad():
            off = 0
            for p in self.model.parameters():
                n = p.numel()
                p.copy_(flat[off:off + n].view_as(p))
                off += n
        return self.model

    def optimizer_state_dict(self) -> Dict[str, Any]:
        return flat_to_adam_state(self.exp_avg, self.exp_avg_sq, self.segments, self.global_steps, self.lr,
                                  self.betas, self.eps, self.weight_decay, self.adamw)

    # ---- ZeRO-1: each rank's optimizer state is current only on the elements it owns
    @property
    def _sharded_ckpt(self) -> bool:
        return self.zero_stage == 1  # DeepSpeed writes zero_pp_rank shards at any world size

    def _owned_index(self) -> torch.Tensor:
        own = zero1_owner_map(self.F, self.H, self.world_size)
        return torch.nonzero(own == self.rank).reshape(-1)

    def _gather_zero1_moments(self) -> None:
        """Replicate the moments from their owners (each rank contributes its owned elements): the
        state a replicated (ZeRO-0-math) path needs after the sharded fused kernel."""
        own = zero1_owner_map(self.F, self.H, self.world_size)
        mask = torch.zeros(self.padded, dtype=torch.float32)
        mask[: self.numel] = (own == self.rank).float()
        mask = mask.to(self.device)
        for t in (self.exp_avg, self.exp_avg_sq):
            t.mul_(mask)
            comm.all_reduce_(t)

    def _zero_shard(self) -> Dict[str, Any]:
        idx = self._owned_index()
        idx_d = idx.to(self.device)
        return {
            "zero_stage": 1,
            "partition_rank": self.rank,
            "partition_world_size": self.world_size,
            "index": idx,  # owned flat elements (the fused kernel's lane ownership, zero1_owner_map)
            "total": self.numel,
            "names": [n for n, _, _ in simple_net_layout(self.F, self.H)],
            "offsets": [o for _, _, o in simple_net_layout(self.F, self.H)],
            "shapes": [list(shp) for _, shp, _ in simple_net_layout(self.F, self.H)],
            "fp32_flat": self.params[idx_d].detach().cpu().clone(),
            "exp_avg": self.exp_avg[idx_d].detach().cpu().clone(),
            "exp_avg_sq": self.exp_avg_sq[idx_d].detach().cpu().clone(),
            "step": self.global_steps,
            "param_groups": [{"lr": self.lr, "betas": list(self.betas), "eps": self.eps,
                              "weight_decay": self.weight_decay, "adamw": self.adamw}],
        }

    def save_checkpoint(self, save_dir: str, tag: Optional[str] = None, client_state: Optional[dict] = None) -> str:
        self.sync_model()
        shard = self._zero_shard() if self._sharded_ckpt else None
        return ckpt.save(save_dir, tag, self.global_steps,
                         {k: v.detach().cpu().clone() for k, v in self.model.state_dict().items()},
                         None if shard is not None else self.optimizer_state_dict(),
                         {"global_samples": self.global_samples, "dp_world_size": self.world_size,
                          "client_state": client_state or {}},
                         self.ds_config, zero_shard=shard)

    def load_checkpoint(self, load_dir: str, tag: Optional[str] = None, load_optimizer_states: bool = True):
        path, states, shard = ckpt.load(load_dir, tag)
        if states is None:
            return None, None
        self.model.load_state_dict(states["module"])
        self.params[: self.numel].copy_(pack_simple_net(self.model).to(self.device))
        self.global_steps = int(states.get("global_steps", 0))
        if load_optimizer_states and self._sharded_ckpt:
            if shard is None or "index" not in shard:
                raise FileNotFoundError(f"missing fused-kernel ZeRO-1 shard for rank {self.rank} under {path}")
            if int(shard["partition_world_size"]) != self.world_size or int(shard["total"]) != self.numel:
                raise RuntimeError("ZeRO-1 checkpoint was written with a different world size / model; "
                                   "consolidate it with zero_to_fp32.py and load the fp32 weights instead")
            idx = shard["index"].to(self.device)
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            self.exp_avg[idx] = shard["exp_avg"].to(self.device)
            self.exp_avg_sq[idx] = shard["exp_avg_sq"].to(self.device)
            if not (self.zero1 and self.impl == "fused"):
                self._gather_zero1_moments()  # a replicated path needs every element's moments
        elif load_optimizer_states and states.get("optimizer"):
            step = adam_state_to_flat(states["optimizer"], self.exp_avg, self.exp_avg_sq, self.segments)
            self.global_steps = int(states.get("global_steps", step))
        self.global_samples = int(states.get("global_samples", 0))
        return path, states.get("client_state", {})

    def close_graph_resources(self) -> None:
        if self.rccl is not None:
            self.rccl.close()
            self.rccl = None
        self._graph = None

    def close(self) -> None:
        self._drop_launcher()  # holds the mailbox pointers: before the channel goes
        if self.channel is not None:
            self.channel.close()
            self.channel = None
        if self.rccl is not None:
            self.rccl.close()
            self.rccl = None
        self._graph = None
