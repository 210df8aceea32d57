"""bf16 trainer for the bench-size synthetic MLP on the HIP MFMA GEMM (``csrc/gemm.hip``).

Reference: the loop of ``train.py:98-117`` on a bench-size ``SimpleNet`` (``train.py:26-36``).

One optimizer step, all on the GPU, no host sync:

    forward   a_l = relu(a_{l-1} W_l^T + b_l)   gemm_nt epilogue: bias + ReLU + bf16 a_l and a_l^T
    head      z = a_L w + b, BCE, dz, g_L = dz w^T * 1[a_L > 0] (+ g_L^T), dw, db      (mlp_head)
    backward  dW_l = g_l^T a_{l-1}   -> bf16 (or fp32) gradient buffer                  (gemm_nt)
              g_{l-1} = (g_l W_l) * 1[a_{l-1} > 0] (+ g_{l-1}^T)   epilogue: mask  (gemm_nt, b_kn)
                        + per-128-row-tile column sums of g_{l-1}: db_{l-1} partials (colsum)
              db_l, head dw: ONE fixed-order reduction of the partials (partials_reduce_multi)
              each layer's weight gradient leaves for its collective as soon as its wgrad is
              enqueued (RCCL over xGMI on the process group's stream): the collective overlaps
              the remaining backward GEMMs
    update    fused Adam over the fp32 masters that also writes the bf16 compute copy (ZeRO-1: on
              the shard, then all-gather); the dgrad GEMM reads W_l[out, in] directly (a [K, N]
              operand through gfx950 transposed LDS reads), so no transposed weight copy exists

Schedules (``schedule=`` or ``DGT_MLP_SCHEDULE``):

* ``"flat"``: after backward, ONE Adam launch over every weight (one rank, opt-in
  ``fuse_adam=True`` / ``DGT_MLP_FUSED_ADAM=1``: each layer's wgrad GEMM applies Adam in its
  epilogue instead, ``gemm_nt_adam_``, so no gradient reaches memory -- measured slower in round 3:
  the epilogue streams the optimizer state at ~4.8 TB/s from one 8-wave block per CU, the flat
  launch at ~5.6 TB/s, 1,153-1,168 vs 1,233-1,281 iters/s, profiles/r3_mlp_fused_vs_flat_adam.txt);
* ``"overlap"`` (default for N > 1): layer l's update runs on a side HIP stream as soon as its
  collective has landed and backward no longer reads W_l, so the Adam of the upper layers
  overlaps the collectives of the lower ones and only the first layer's update is left after
  the last collective; the next step's forward GEMM of layer l waits only on layer l's event;
* ``"serial"``: the same per-layer updates on the main stream after backward.

On one GPU the overlap does not pay: a streaming Adam running beside the backward GEMMs slows
them by as much as it hides (dgrad 49 -> 70 us, profiles/r1_mlp_schedule_ab.txt) — the GEMMs at
M = 1024 are bound by the L2/fabric, not by MFMA.  (The round-1/2 A/B switches -- a refreshed W^T
for the dgrad, an Adam kernel writing W and W^T, a side-stream wgrad + Adam, GEMM variants -- were
measured slower or no better and removed; their records stay in profiles/.)

Parameters live in two flat regions:

* the big region — the L weight matrices, bf16 for compute + gradients (bf16 by default, as
  PyTorch autocast's matmul backward produces them: half the wgrad store, Adam read and
  collective bytes; ``grad_dtype=torch.float32`` / ``DGT_MLP_GRAD_DTYPE=fp32`` keeps fp32), each
  matrix padded to a multiple of 64 * world_size elements (a per-layer communication bucket).
  The collectives carry the gradient buffer itself, so the wire dtype IS the gradient dtype:
  ``comm_dtype=torch.float32`` (DeepSpeed's ``communication_data_type``) selects fp32 gradients.
  An 8-rank bf16 sum adds 3.7e-3 relative RMS error against 1.7e-3 for the bf16 rounding of
  the gradient itself (tests/test_multiproc_cpu.py::test_bf16_gradient_wire_error_eight_ranks),
  so bf16 stays the default wire;
* the small region — biases and the head, fp32 (the GEMM epilogues read fp32 biases), replicated
  on every rank and all-reduced as one bucket.

Checkpoints (``save_checkpoint`` / ``load_checkpoint``) use the DeepSpeed layout of
``runtime/checkpoint.py``: the module's fp32 weights and, for ZeRO-0, the Adam state in torch's
per-parameter format in ``mp_rank_00_model_states.pt``; for ZeRO-1 each rank's fp32 master and
moment shards of the weight buckets in ``zero_pp_rank_{r}_mp_rank_00_optim_states.pt`` (bucket
format, so ``zero_to_fp32.py`` consolidates them), with the replicated small region alongside.

``zero_stage=0``: every rank keeps the full fp32 master of the big region; its buckets are
all-reduced and one Adam launch updates everything.  ``zero_stage=1`` (DeepSpeed ZeRO-1/2 for the
matrices): each bucket is REDUCE-SCATTERED into this rank's gradient shard, Adam updates
only the 1/N master shard (N x less optimizer traffic and memory), and the bf16 parameter shards
are ALL-GATHERED back: one reduce-scatter + one all-gather pass on the wire per parameter, the
same bytes as an all-reduce, with 1/N of the Adam traffic.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import contextlib
import os

import torch
import torch.distributed as dist

from ..accelerator import get_accelerator
from ..models.synthetic_mlp import SyntheticMLP, synthetic_batch_data
from ..ops.adam import adam_flat_
from ..ops.gemm import gemm_nt, gemm_nt_adam_, mlp_head, partials_reduce_multi, rowsum_bf16, transpose_bf16
from ..parallel import comm
from . import checkpoint as ckpt

ALIGN = 64
SCHEDULES = ("overlap", "serial", "flat")


def _round(x: int, m: int = ALIGN) -> int:
    return (x + m - 1) // m * m


class MLPTrainer:
    impl = "hip-mfma-bf16"

    def __init__(self, model: SyntheticMLP, batch_size: int = 1024, n_batches: int = 8, lr: float = 1e-4,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, seed: int = 1234,
                 device: Optional[torch.device] = None, zero_stage: int = 0, schedule: Optional[str] = None,
                 grad_dtype: Optional[torch.dtype] = None, comm_dtype: Optional[torch.dtype] = None,
                 fuse_adam: Optional[bool] = None, bucket_mb: Optional[float] = None):
        if zero_stage not in (0, 1):
            raise ValueError("MLPTrainer supports zero_stage 0 or 1")
        if comm_dtype not in (None, torch.bfloat16, torch.float32):
            raise ValueError("comm_dtype must be torch.bfloat16 or torch.float32")
        if grad_dtype is None:
            grad_dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[os.environ.get("DGT_MLP_GRAD_DTYPE", "bf16")]
        if comm_dtype is not None and comm_dtype != grad_dtype:
            # DeepSpeed's communication_data_type: the collectives carry the gradient buffer itself,
            # so an fp32 wire means fp32 gradients straight out of the wgrad epilogue (no cast pass);
            # a bf16 wire with fp32 gradients would only add rounding
            grad_dtype = comm_dtype
        if grad_dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("grad_dtype must be torch.bfloat16 or torch.float32")
        self.grad_dtype = grad_dtype
        schedule = schedule or os.environ.get("DGT_MLP_SCHEDULE", "auto")
        if schedule not in SCHEDULES + ("auto",):
            raise ValueError(f"schedule must be one of {SCHEDULES} or 'auto'")
        if schedule == "auto":  # measured (profiles/r1_mlp_schedule_ab.txt): see the module docstring
            schedule = "flat" if comm.get_world_size() == 1 else "overlap"
        self.device = device or get_accelerator().device()
        self.model = model
        self.B, self.D, self.L, self.Din = batch_size, model.width, model.depth, model.in_features
        self.rank, self.world_size = comm.get_rank(), comm.get_world_size()
        # collectives run at N > 1, or at N = 1 under DGT_FORCE_COLLECTIVES (same code, 1-rank RCCL)
        self.coll = comm.collectives_on(self.world_size)
        self.zero_stage = zero_stage if self.coll else 0
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.global_steps = 0
        dev, ws = self.device, self.world_size
        named = dict(model.named_parameters())

        # ---- big region: W_l, each padded to a multiple of ALIGN * world_size (one bucket each)
        self.w_off: List[int] = []
        self.w_len: List[int] = []
        off = 0
        for i in range(self.L):
            self.w_off.append(off)
            self.w_len.append(_round(named[f"layers.{i}.weight"].numel(), ALIGN * ws))
            off += self.w_len[-1]
        self.total_w = off
        w_full = torch.zeros(self.total_w, dtype=torch.float32)
        for i in range(self.L):
            p = named[f"layers.{i}.weight"]
            w_full[self.w_off[i]:self.w_off[i] + p.numel()] = p.detach().reshape(-1).float()
        # ---- small region: b_l, head.weight, head.bias (fp32, replicated)
        self.s_off: Dict[str, int] = {}
        off = 0
        for name in [f"layers.{i}.bias" for i in range(self.L)] + ["head.weight", "head.bias"]:
            self.s_off[name] = off
            off = _round(off + named[name].numel())
        self.total_s = off
        s_full = torch.zeros(self.total_s, dtype=torch.float32)
        for name, o in self.s_off.items():
            s_full[o:o + named[name].numel()] = named[name].detach().reshape(-1).float()
        w_full, s_full = w_full.to(dev), s_full.to(dev)
        comm.broadcast_(w_full, 0)  # DeepSpeed _broadcast_model
        comm.broadcast_(s_full, 0)

        self.params_bf16 = w_full.to(torch.bfloat16)  # compute copy of every W_l
        self.grads_w = torch.zeros(self.total_w, dtype=grad_dtype, device=dev)
        self.master_s = s_full
        self.grads_s = torch.zeros_like(self.master_s)
        self.m_s, self.v_s = torch.zeros_like(self.master_s), torch.zeros_like(self.master_s)
        if self.zero_stage == 0:
            self.master_w = w_full
            self.lp_w = self.params_bf16
            self.shard_grad = None
            self.shard_len = list(self.w_len)
            self.shard_off = list(self.w_off)
        else:  # this rank's 1/N of every bucket, concatenated
            self.shard_len = [n // ws for n in self.w_len]
            self.shard_off = [sum(self.shard_len[:i]) for i in range(self.L)]
            pieces = [w_full[self.w_off[i] + self.rank * n:self.w_off[i] + (self.rank + 1) * n]
                      for i, n in enumerate(self.shard_len)]
            self.master_w = torch.cat(pieces).contiguous()
            self.lp_w = torch.empty(self.master_w.numel(), dtype=torch.bfloat16, device=dev)
            self.shard_grad = torch.zeros(self.master_w.numel(), dtype=grad_dtype, device=dev)
            del w_full
        self.m_w, self.v_w = torch.zeros_like(self.master_w), torch.zeros_like(self.master_w)
        self._plan_buckets(bucket_mb)

        def wview(buf, i):
            shape = named[f"layers.{i}.weight"].shape
            return buf[self.w_off[i]:self.w_off[i] + shape[0] * shape[1]].view(shape)

        def sview(buf, name):
            o = self.s_off[name]
            return buf[o:o + named[name].numel()]

        self.W = [wview(self.params_bf16, i) for i in range(self.L)]
        self.gW = [wview(self.grads_w, i) for i in range(self.L)]
        self.b = [sview(self.master_s, f"layers.{i}.bias") for i in range(self.L)]
        self.gb = [sview(self.grads_s, f"layers.{i}.bias") for i in range(self.L)]
        self.hw, self.hb = sview(self.master_s, "head.weight"), sview(self.master_s, "head.bias")
        self.ghw, self.ghb = sview(self.grads_s, "head.weight"), sview(self.grads_s, "head.bias")
        # dgrad g_{l-1} = g_l . W_l: the GEMM reads W_l[out, in] as a [K, N] operand through
        # transposed LDS reads (gemm_nt(..., b_kn=True)), so no W^T exists at all
        # single rank, ZeRO-0, opt-in: nothing reduces the weight gradients, so each wgrad GEMM can
        # apply Adam to its tile in its epilogue (gemm_nt_adam_) and no gradient reaches memory
        if fuse_adam is None:  # measured: the flat Adam launch wins (module docstring)
            fuse_adam = os.environ.get("DGT_MLP_FUSED_ADAM", "0") == "1"
        self.fused_adam = bool(fuse_adam and dev.type == "cuda" and not self.coll and self.zero_stage == 0)

        # ---- activations (both layouts) and gradient scratch
        B, D = self.B, self.D
        self.a = [None] + [torch.empty(B, D, dtype=torch.bfloat16, device=dev) for _ in range(self.L)]
        self.aT = [None] + [torch.empty(D, B, dtype=torch.bfloat16, device=dev) for _ in range(self.L)]
        # three gradient buffers: with the side-stream wgrad+Adam (below) a layer's g^T is still being
        # read while the next two dgrads write theirs
        self.g = [torch.empty(B, D, dtype=torch.bfloat16, device=dev) for _ in range(3)]
        self.gT = [torch.empty(D, B, dtype=torch.bfloat16, device=dev) for _ in range(3)]
        self.dz = torch.empty(B, dtype=torch.float32, device=dev)
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=dev)
        # bias-gradient and head-dw partials: the dgrad epilogue leaves per-128-row-tile column sums
        # of g_{l-1} (colsum), the head per-64-row-tile sums of g_{L-1} and of dz a; ONE fixed-order
        # reduction launch after backward turns them into the small region's gradients (instead of
        # a row-sum launch per layer and the head's own reduction)
        # (the GPU kernels need B % 128 == 0 anyway; a CPU run with another batch takes per-layer row sums)
        self._partials = B % 128 == 0
        self.bpart = [torch.empty(B // 128, D, dtype=torch.float32, device=dev) if self._partials else None
                      for _ in range(self.L - 1)]
        self.bpart_top = torch.empty(B // 64, D, dtype=torch.float32, device=dev) if self._partials else None
        self.hw_part = torch.empty(B // 64, D, dtype=torch.float32, device=dev) if self._partials else None

        # ---- synthetic data (different stream per rank: weak-scaling data parallelism)
        n = B * n_batches
        x, y = synthetic_batch_data(n, self.Din, seed + self.rank)
        self.X = x.to(dev, torch.bfloat16)
        self.XT = torch.empty(self.Din, n, dtype=torch.bfloat16, device=dev)
        transpose_bf16(self.X, self.XT)
        self.Y = y.to(dev)
        self.n_batches = n_batches
        kind = "allreduce" if self.zero_stage == 0 else "reducescatter+allgather"
        self.exchange = f"{comm.backend_name()}-{kind}-per-layer" if self.coll else "none"

        # ---- schedule: side streams + per-layer events (GPU only; CPU runs everything in order)
        self.schedule = schedule if dev.type == "cuda" else "serial"
        self.shapes = [tuple(named[f"layers.{i}.weight"].shape) for i in range(self.L)]
        self._overlap = self.schedule == "overlap"
        self._opt_pending = False
        self.s_main = None
        # A/B knobs of the fused single-rank step: the wgrad+Adam launches on a side stream beside the
        # dgrads (DGT_MLP_WGA_SIDE=1), and the GEMM variant of each product (ops/gemm.py gemm_nt:
        # 1 = 128x128 2-stage, 64 KiB of LDS, so two different kernels' blocks can share a CU)
        self._wga_side = (dev.type == "cuda" and os.environ.get("DGT_MLP_WGA_SIDE", "0") == "1")
        self._v_wga = int(os.environ.get("DGT_MLP_WGA_VARIANT", "0") or 0)
        self._v_dgrad = int(os.environ.get("DGT_MLP_DGRAD_VARIANT", "0") or 0)
        self._v_fwd = int(os.environ.get("DGT_MLP_FWD_VARIANT", "0") or 0)
        self._v_wgrad = int(os.environ.get("DGT_MLP_WGRAD_VARIANT", "0") or 0)
        if self._wga_side:
            from ..accelerator import concurrent_stream  # (its own hardware queue: see the overlap schedule)
            self.s_opt = concurrent_stream(dev, slot=2)[0]
            self.ev_bwd = [torch.cuda.Event() for _ in range(self.L)]
            self.ev_opt = [torch.cuda.Event() for _ in range(self.L)]
        if self._overlap:
            # side streams measured to sit on hardware queues other than the compute stream's (two
            # streams on one queue run in turn: accelerator.concurrent_stream)
            from ..accelerator import concurrent_stream
            self.s_comm = concurrent_stream(dev, slot=1)[0]
            self.s_opt = concurrent_stream(dev, slot=2)[0]
            self.ev_wgrad = [torch.cuda.Event() for _ in range(self.L)]
            self.ev_bwd = [torch.cuda.Event() for _ in range(self.L)]
            self.ev_comm = [torch.cuda.Event() for _ in range(self.L)]
            self.ev_opt = [torch.cuda.Event() for _ in range(self.L)]

    # ------------------------------------------------------------------ helpers
    def _plan_buckets(self, bucket_mb: Optional[float]) -> None:
        """The weight region's communication buckets (``bucket_mb`` / ``DGT_MLP_BUCKET_MB``).

        Default (None): one bucket per layer matrix (33.5 MB bf16 at width 4096).  With a size, the
        region is cut into contiguous pieces of that many MiB from its top (the last layer's end,
        where backward starts), each a multiple of ALIGN x world_size elements: a layer larger than
        the size leaves in several collectives, smaller layers share one.  A bucket leaves once the
        wgrad of the lowest layer it touches is enqueued (``bucket_ready[i]``: buckets issued after
        layer i's wgrad), and layer i's update waits for the last bucket covering it
        (``update_after[i]``: the backward iteration that issues it).  ZeRO-1 keeps per-layer
        buckets (its shards are per layer)."""
        if bucket_mb is None and os.environ.get("DGT_MLP_BUCKET_MB"):
            bucket_mb = float(os.environ["DGT_MLP_BUCKET_MB"])
        L, esize = self.L, (2 if self.grad_dtype == torch.bfloat16 else 4)
        quantum = ALIGN * self.world_size
        if bucket_mb is None or self.zero_stage == 1:
            self.bucket_mb = None
            spans = [(self.w_off[i], self.w_off[i] + self.w_len[i]) for i in reversed(range(L))]
        else:
            if bucket_mb <= 0:
                raise ValueError("bucket_mb must be positive")
            self.bucket_mb = float(bucket_mb)
            cap = max(quantum, int(bucket_mb * (1 << 20)) // esize // quantum * quantum)
            spans, hi = [], self.total_w
            while hi > 0:
                spans.append((max(0, hi - cap), hi))
                hi = spans[-1][0]

        def layer_of(e: int) -> int:
            return max(i for i in range(L) if self.w_off[i] <= e)

        self.buckets = spans  # in issue order (descending memory = backward order)
        self.bucket_ready: List[List[int]] = [[] for _ in range(L)]
        for b, (lo, _) in enumerate(spans):
            self.bucket_ready[layer_of(lo)].append(b)
        # layer i is complete once the bucket holding its lowest element has been reduced
        self.update_after = [layer_of(next(lo for lo, hi in spans if lo <= self.w_off[i] < hi)) for i in range(L)]

    def flops_per_step(self) -> int:
        return self.model.flops_per_sample() * self.B

    def grad_of(self, name: str) -> torch.Tensor:
        """This rank's local (pre-reduction) gradient of a model parameter, in its shape."""
        if self.fused_adam and name.startswith("layers.") and name.endswith("weight"):
            raise RuntimeError("weight gradients are consumed in place by the fused wgrad+Adam; "
                               "construct MLPTrainer(fuse_adam=False) to inspect them")
        self.join()
        p = dict(self.model.named_parameters())[name]
        if name.startswith("layers.") and name.endswith("weight"):
            return self.gW[int(name.split(".")[1])].reshape(p.shape)
        o = self.s_off[name]
        return self.grads_s[o:o + p.numel()].reshape(p.shape)

    @staticmethod
    def _collective(fn, out: torch.Tensor, *inp: torch.Tensor, works: list) -> None:
        if comm.needs_host_staging(out):  # gloo rehearsal with GPU tensors: via host memory
            host_out = out.detach().cpu()
            fn(host_out, *[t.detach().cpu() for t in inp])
            out.copy_(host_out)
        else:
            works.append(fn(out, *inp, async_op=True))

    def _reduce_layer(self, i: int, works: list) -> None:
        """The collectives of the buckets that become ready with layer i's wgrad."""
        if not self.coll:
            return
        if self.zero_stage == 0:
            for b in self.bucket_ready[i]:
                lo, hi = self.buckets[b]
                self._collective(dist.all_reduce, self.grads_w[lo:hi], works=works)
        else:
            bucket = self.grads_w[self.w_off[i]:self.w_off[i] + self.w_len[i]]
            out = self.shard_grad[self.shard_off[i]:self.shard_off[i] + self.shard_len[i]]
            self._collective(dist.reduce_scatter_tensor, out, bucket, works=works)

    def _allgather_params(self) -> None:
        works: list = []
        for i in range(self.L):
            out = self.params_bf16[self.w_off[i]:self.w_off[i] + self.w_len[i]]
            piece = self.lp_w[self.shard_off[i]:self.shard_off[i] + self.shard_len[i]]
            self._collective(dist.all_gather_into_tensor, out, piece, works=works)
        for w in works:
            w.wait()

    # ------------------------------------------------------------------ optimizer pieces
    def _adam_args(self):
        return (self.global_steps, self.lr, self.betas[0], self.betas[1], self.eps, self.weight_decay, False)

    def _update_layer(self, i: int) -> None:
        """Adam on layer i's weights (its shard under ZeRO-1) + refresh of the bf16 W_i."""
        args, scale = self._adam_args(), 1.0 / self.world_size
        if self.zero_stage == 0:
            o = self.w_off[i]
            sl = slice(o, o + self.w_len[i])
            adam_flat_(self.master_w[sl], self.grads_w[sl], self.m_w[sl], self.v_w[sl], *args, grad_scale=scale,
                       param_lp=self.params_bf16[sl])
        else:
            sl = slice(self.shard_off[i], self.shard_off[i] + self.shard_len[i])
            adam_flat_(self.master_w[sl], self.shard_grad[sl], self.m_w[sl], self.v_w[sl], *args, grad_scale=scale,
                       param_lp=self.lp_w[sl])
            works: list = []
            out = self.params_bf16[self.w_off[i]:self.w_off[i] + self.w_len[i]]
            self._collective(dist.all_gather_into_tensor, out, self.lp_w[sl], works=works)
            for w in works:
                w.wait()

    def join(self) -> None:
        """Make the caller's stream wait for the side streams (results visible to later work)."""
        if self._opt_pending:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_stream(self.s_opt)
            if self._overlap:
                cur.wait_stream(self.s_comm)
            self._opt_pending = False

    # ------------------------------------------------------------------ one step
    def step(self, s: int) -> None:
        B, L = self.B, self.L
        j = s % self.n_batches
        x = self.X[j * B:(j + 1) * B]
        xT = self.XT[:, j * B:(j + 1) * B]
        y = self.Y[j * B:(j + 1) * B]
        ov = self._overlap
        main = torch.cuda.current_stream(self.device) if (ov or self._wga_side) else None
        # forward: layer i waits only on its own update of the previous step (and, on the side
        # stream, every later layer's, which read aT[i + 1] and were enqueued first)
        prev = x
        for i in range(L):
            if self._opt_pending:
                main.wait_event(self.ev_opt[i])
            # a_{i+1}^T feeds the wgrad of layer i+1: the last layer's output has none (the head reads a_L)
            gemm_nt(prev, self.W[i], C=self.a[i + 1], CT=self.aT[i + 1] if i + 1 < L else None, bias=self.b[i],
                    relu=True, variant=self._v_fwd)
            prev = self.a[i + 1]
        # head (+ its gradients, written in place: no zero fills)
        cur = 0
        mlp_head(self.a[L], self.hw, self.hb, y, self.dz, self.ghw, self.ghb, self.loss_acc, self.g[cur],
                 self.gT[cur], dw_part=self.hw_part, bias_part=self.bpart_top)
        self.global_steps += 1
        if self.fused_adam:
            self._backward_fused_adam(xT, cur)
            return
        works: list = []
        # backward, last layer first; each weight bucket leaves for its collective as soon as its
        # wgrad is enqueued; with the overlap schedule the layer's optimizer update follows on
        # s_opt once backward no longer reads W_i^T (after its dgrad) and the collective is done
        for i in reversed(range(L)):
            a_prevT = xT if i == 0 else self.aT[i]
            # (a side stream running this wgrad beside the same layer's dgrad measured 8 % slower per
            # step: two one-wave grids of one-block-per-CU kernels compete for the CUs,
            # profiles/r4_mlp_wgrad_side_ab.txt)
            gemm_nt(self.gT[cur], a_prevT, C=self.gW[i], out_f32=self.grad_dtype == torch.float32,
                    variant=self._v_wgrad)
            if not self._partials:
                rowsum_bf16(self.gT[cur], self.gb[i])
            if self.coll:
                if ov:
                    self.ev_wgrad[i].record(main)
                    self.s_comm.wait_event(self.ev_wgrad[i])
                    with torch.cuda.stream(self.s_comm):
                        lw: list = []
                        self._reduce_layer(i, lw)
                        for w in lw:
                            w.wait()
                        self.ev_comm[i].record(self.s_comm)
                else:
                    self._reduce_layer(i, works)
            if i > 0:
                # g_{i-1} row-major feeds the next dgrad only: the last one (i == 1) writes just g_0^T
                gemm_nt(self.g[cur], self.W[i], C=self.g[cur ^ 1] if i > 1 else None, CT=self.gT[cur ^ 1],
                        mask=self.a[i], b_kn=True, variant=self._v_dgrad, colsum=self.bpart[i - 1])
                cur ^= 1
            if ov:
                self.ev_bwd[i].record(main)
                # the layers whose last bucket left at this iteration (per-layer buckets: layer i);
                # their dgrads (which read W) ran at iterations >= i, all enqueued before ev_bwd[i]
                for u in reversed(range(i, L)):
                    if self.update_after[u] != i:
                        continue
                    self.s_opt.wait_event(self.ev_bwd[i])
                    if self.coll:
                        self.s_opt.wait_event(self.ev_comm[i])
                    with torch.cuda.stream(self.s_opt):
                        self._update_layer(u)
                        self.ev_opt[u].record(self.s_opt)
        small_done = self._reduce_small(with_adam=True)
        if self.coll:  # biases + head: one small replicated bucket
            self._collective(dist.all_reduce, self.grads_s, works=works)
        for w in works:
            w.wait()
        if not small_done:
            adam_flat_(self.master_s, self.grads_s, self.m_s, self.v_s, *self._adam_args(),
                       grad_scale=1.0 / self.world_size)
        if ov:
            self._opt_pending = True
        elif self.schedule == "serial":
            for i in reversed(range(L)):
                self._update_layer(i)
        else:  # "flat": one Adam launch over every weight, then the all-gather
            grads_w = self.grads_w if self.zero_stage == 0 else self.shard_grad
            adam_flat_(self.master_w, grads_w, self.m_w, self.v_w, *self._adam_args(),
                       grad_scale=1.0 / self.world_size, param_lp=self.lp_w)
            if self.zero_stage == 1:
                self._allgather_params()

    def _reduce_small(self, with_adam: bool = False) -> bool:
        """The small region's gradients from their partials, in one launch: every hidden bias (the
        dgrads' and the head's column sums of g) and the head weight (the head's dz a partials).
        ``with_adam`` (one rank, GPU): the same launch also applies the region's Adam step -- the head
        bias (written by the head itself, padded to 4) rides along as a one-tile segment -- and
        True is returned (the caller skips its adam_flat over the region)."""
        L = self.L
        if not self._partials:
            return False
        pairs = ([(self.bpart_top, self.gb[L - 1])] + [(self.bpart[i], self.gb[i]) for i in range(L - 1)]
                 + [(self.hw_part, self.ghw)])
        fuse = with_adam and self.device.type == "cuda" and not self.coll
        if fuse:
            o = self.s_off["head.bias"]
            hb4 = self.grads_s[o:o + 4]  # the head bias and three padding zeros (never written)
            pairs.append((hb4.view(1, 4), hb4))
            partials_reduce_multi(pairs, adam=(self.grads_s, self.master_s, self.m_s, self.v_s, *self._adam_args(),
                                               1.0 / self.world_size))
            return True
        partials_reduce_multi(pairs)
        return False

    def _backward_fused_adam(self, xT: torch.Tensor, cur: int) -> None:
        """Single-rank backward + update: per layer, the bias-gradient row sums, the dgrad (it
        reads W_l, so it runs BEFORE W_l changes), then ONE launch that computes dW_l and applies
        Adam to W_l in its epilogue (fp32 master / moments + the bf16 compute copy).  The weight
        region moves 26 B/param (12 read + 14 written) instead of the wgrad store + flat Adam's
        2 + 28 B/param, and the update overlaps the other blocks' MFMA work."""
        args = self._adam_args()
        side = self._wga_side
        main = torch.cuda.current_stream(self.device) if side else None
        for i in reversed(range(self.L)):
            a_prevT = xT if i == 0 else self.aT[i]
            nxt = (cur + 1) % 3
            if not self._partials:
                rowsum_bf16(self.gT[cur], self.gb[i])
            if side and i + 2 < self.L:
                # the buffers rotate mod 3: this dgrad writes gT[nxt], which layer i + 2's side-stream
                # wgrad + Adam may still be reading (WAR); wait for that update first
                main.wait_event(self.ev_opt[i + 2])
            if i > 0:
                gemm_nt(self.g[cur], self.W[i], C=self.g[nxt] if i > 1 else None, CT=self.gT[nxt], mask=self.a[i],
                        b_kn=True, variant=self._v_dgrad, colsum=self.bpart[i - 1])
            R, Cc = self.shapes[i]
            sl = slice(self.w_off[i], self.w_off[i] + R * Cc)
            if side:  # after the dgrad (it read W_i) and with gT[cur] complete
                self.ev_bwd[i].record(main)
                self.s_opt.wait_event(self.ev_bwd[i])
            with torch.cuda.stream(self.s_opt) if side else contextlib.nullcontext():
                gemm_nt_adam_(self.gT[cur], a_prevT, self.master_w[sl].view(R, Cc), self.m_w[sl].view(R, Cc),
                              self.v_w[sl].view(R, Cc), self.params_bf16[sl].view(R, Cc), *args,
                              grad_scale=1.0 / self.world_size, variant=self._v_wga)
                if side:
                    self.ev_opt[i].record(self.s_opt)
            if i > 0:
                cur = nxt
        self._reduce_small()
        adam_flat_(self.master_s, self.grads_s, self.m_s, self.v_s, *args, grad_scale=1.0 / self.world_size)
        if side:
            self._opt_pending = True

    # ------------------------------------------------------------------ checkpoints
    def _param_names(self) -> List[str]:
        return [n for n, _ in self.model.named_parameters()]

    def _full_fp32(self, name: str) -> torch.Tensor:
        """A parameter's current fp32 value (the master where this rank holds it whole)."""
        p = dict(self.model.named_parameters())[name]
        if name.startswith("layers.") and name.endswith("weight"):
            i = int(name.split(".")[1])
            src = self.master_w if self.zero_stage == 0 else self.params_bf16
            return src[self.w_off[i]:self.w_off[i] + p.numel()].float().view(p.shape)
        o = self.s_off[name]
        return self.master_s[o:o + p.numel()].view(p.shape)

    def _moments(self, name: str):
        p = dict(self.model.named_parameters())[name]
        if name.startswith("layers.") and name.endswith("weight"):
            i = int(name.split(".")[1])
            o = self.w_off[i]
            return self.m_w[o:o + p.numel()].view(p.shape), self.v_w[o:o + p.numel()].view(p.shape)
        o = self.s_off[name]
        return self.m_s[o:o + p.numel()].view(p.shape), self.v_s[o:o + p.numel()].view(p.shape)

    def _zero_shard(self) -> Dict:
        names = [f"layers.{i}.weight" for i in range(self.L)]
        return {
            "zero_stage": 1,
            "partition_rank": self.rank,
            "partition_world_size": self.world_size,
            "buckets": [[self.w_off[i], self.w_len[i]] for i in range(self.L)],
            "offsets": list(self.w_off),
            "shapes": [list(self.shapes[i]) for i in range(self.L)],
            "names": names,
            "total": self.total_w,
            "fp32_flat": self.master_w.detach().cpu().clone(),
            "exp_avg": self.m_w.detach().cpu().clone(),
            "exp_avg_sq": self.v_w.detach().cpu().clone(),
            "small": {"master": self.master_s.detach().cpu().clone(), "exp_avg": self.m_s.detach().cpu().clone(),
                      "exp_avg_sq": self.v_s.detach().cpu().clone(), "offsets": dict(self.s_off)},
            "step": self.global_steps,
            "param_groups": [{"lr": self.lr, "betas": list(self.betas), "eps": self.eps,
                              "weight_decay": self.weight_decay, "adamw": False}],
        }

    def save_checkpoint(self, save_dir: str, tag: Optional[str] = None, client_state: Optional[dict] = None,
                        ds_config: Optional[dict] = None) -> str:
        """DeepSpeed-layout checkpoint of the current step (see the module docstring)."""
        self.join()
        names = self._param_names()
        module = {n: self._full_fp32(n).detach().cpu().clone() for n in names}
        optimizer = None
        if self.zero_stage == 0:
            state = {}
            if self.global_steps > 0:
                for i, n in enumerate(names):
                    m, v = self._moments(n)
                    state[i] = {"step": torch.tensor(float(self.global_steps)), "exp_avg": m.detach().cpu().clone(),
                                "exp_avg_sq": v.detach().cpu().clone()}
            optimizer = {"state": state, "param_groups": [{
                "lr": self.lr, "betas": tuple(self.betas), "eps": self.eps, "weight_decay": self.weight_decay,
                "amsgrad": False, "maximize": False, "foreach": None, "capturable": False, "differentiable": False,
                "fused": None, "params": list(range(len(names)))}]}
        return ckpt.save(save_dir, tag, self.global_steps, module, optimizer,
                         {"global_samples": self.global_steps * self.B * self.world_size,
                          "dp_world_size": self.world_size, "client_state": client_state or {}},
                         ds_config or {}, zero_shard=self._zero_shard() if self.zero_stage == 1 else None)

    def load_checkpoint(self, load_dir: str, tag: Optional[str] = None, load_optimizer_states: bool = True):
        """Restore masters, bf16 compute copies, moments and the step from ``save_checkpoint``'s layout."""
        path, states, shard = ckpt.load(load_dir, tag)
        if states is None:
            return None, None
        self.join()
        names = self._param_names()
        sd = states["module"]
        dev = self.device
        with torch.no_grad():
            for i in range(self.L):
                w = sd[f"layers.{i}.weight"].reshape(-1).float().to(dev)
                n = w.numel()
                self.params_bf16[self.w_off[i]:self.w_off[i] + n].copy_(w.to(torch.bfloat16))
                if self.zero_stage == 0:
                    self.master_w[self.w_off[i]:self.w_off[i] + n].copy_(w)
            for n in names:
                if n in self.s_off:
                    o = self.s_off[n]
                    v = sd[n].reshape(-1).float().to(dev)
                    self.master_s[o:o + v.numel()].copy_(v)
            self.m_w.zero_(), self.v_w.zero_(), self.m_s.zero_(), self.v_s.zero_()
            if self.zero_stage == 1:
                if shard is None:
                    raise FileNotFoundError(f"missing ZeRO-1 shard for rank {self.rank} under {path}")
                if int(shard["partition_world_size"]) != self.world_size or int(shard["total"]) != self.total_w:
                    raise RuntimeError("ZeRO-1 checkpoint was written with a different world size / model; "
                                       "consolidate it with zero_to_fp32.py and load the fp32 weights instead")
                self.master_w.copy_(shard["fp32_flat"].to(dev))
                self.lp_w.copy_(self.master_w.to(torch.bfloat16))
                if load_optimizer_states:
                    self.m_w.copy_(shard["exp_avg"].to(dev))
                    self.v_w.copy_(shard["exp_avg_sq"].to(dev))
                    self.m_s.copy_(shard["small"]["exp_avg"].to(dev))
                    self.v_s.copy_(shard["small"]["exp_avg_sq"].to(dev))
                self._allgather_params()  # the bf16 compute copy from the exact fp32 shards
            elif load_optimizer_states and states.get("optimizer"):
                st = states["optimizer"]["state"]
                for i, n in enumerate(names):
                    e = st.get(i, st.get(str(i)))
                    if e:
                        m, v = self._moments(n)
                        m.copy_(e["exp_avg"].reshape(m.shape).to(dev))
                        v.copy_(e["exp_avg_sq"].reshape(v.shape).to(dev))
        self.global_steps = int(states.get("global_steps", 0))
        return path, states.get("client_state", {})

    # bench.py adapter (same surface as TinyMLPTrainer)
    def epoch_plan(self, epoch: int):
        plan = torch.arange(self.n_batches, dtype=torch.int32).view(-1, 1)
        return plan, torch.ones(self.n_batches, dtype=torch.int32)

    def run_plan(self, plan, counts) -> None:
        if self.s_main is not None:
            self.s_main.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.s_main):
                for _ in range(int(plan.shape[0])):
                    self.step(self.global_steps)
            torch.cuda.current_stream(self.device).wait_stream(self.s_main)
        else:
            for _ in range(int(plan.shape[0])):
                self.step(self.global_steps)
        self.join()

    @property
    def params(self) -> torch.Tensor:
        """Every parameter as this rank sees it (bf16 matrices + fp32 small params), for checks."""
        self.join()
        return torch.cat([self.params_bf16.float(), self.master_s])

    def check(self) -> None:
        pass

    def close(self) -> None:
        pass
