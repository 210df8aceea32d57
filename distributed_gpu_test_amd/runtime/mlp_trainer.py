"""bf16 trainer for the bench-size synthetic MLP on the HIP MFMA GEMM (``csrc/gemm.hip``).

Reference: the loop of ``train.py:98-117`` on a bench-size ``SimpleNet`` (``train.py:26-36``).

One optimizer step, all on the GPU, no host sync:

    forward   a_l = relu(a_{l-1} W_l^T + b_l)   gemm_nt epilogue: bias + ReLU + bf16 a_l and a_l^T
    head      z = a_L w + b, BCE, dz, g_L = dz w^T * 1[a_L > 0] (+ g_L^T), dw, db      (mlp_head)
    backward  dW_l = g_l^T a_{l-1}   -> fp32 gradient buffer                           (gemm_nt)
              db_l = row sums of g_l^T                                              (rowsum_bf16)
              g_{l-1} = (g_l W_l) * 1[a_{l-1} > 0] (+ g_{l-1}^T)   epilogue: mask      (gemm_nt)
              each layer's weight gradient leaves for its collective as soon as its wgrad is
              enqueued (RCCL over xGMI on the process group's stream): the collective overlaps
              the remaining backward GEMMs
    update    fused Adam launches over flat fp32 masters that also write the bf16 compute copy;
              W_l^T refreshed by a tiled transpose

Parameters live in two flat regions:

* the big region — the L weight matrices, bf16 for compute + fp32 gradients, each matrix padded to
  a multiple of 64 * world_size elements (a per-layer communication bucket);
* the small region — biases and the head, fp32 (the GEMM epilogues read fp32 biases), replicated
  on every rank and all-reduced as one bucket.

``zero_stage=0``: every rank keeps the full fp32 master of the big region; its buckets are
all-reduced and one Adam launch updates everything.  ``zero_stage=1`` (DeepSpeed ZeRO-1/2 for the
matrices): each bucket is REDUCE-SCATTERED into this rank's fp32 gradient shard, Adam updates
only the 1/N master shard (N x less optimizer traffic and memory), and the bf16 parameter shards
are ALL-GATHERED back: 4 + 2 bytes on the wire per parameter instead of an fp32 all-reduce's 8.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..models.synthetic_mlp import SyntheticMLP, synthetic_batch_data
from ..ops.adam import adam_flat_
from ..ops.gemm import gemm_nt, mlp_head, rowsum_bf16, transpose_bf16
from ..parallel import comm

ALIGN = 64


def _round(x: int, m: int = ALIGN) -> int:
    return (x + m - 1) // m * m


class MLPTrainer:
    impl = "hip-mfma-bf16"

    def __init__(self, model: SyntheticMLP, batch_size: int = 1024, n_batches: int = 8, lr: float = 1e-4,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, seed: int = 1234,
                 device: Optional[torch.device] = None, zero_stage: int = 0):
        if zero_stage not in (0, 1):
            raise ValueError("MLPTrainer supports zero_stage 0 or 1")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.model = model
        self.B, self.D, self.L, self.Din = batch_size, model.width, model.depth, model.in_features
        self.rank, self.world_size = comm.get_rank(), comm.get_world_size()
        self.zero_stage = zero_stage if self.world_size > 1 else 0
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
        self.grads_w = torch.zeros(self.total_w, dtype=torch.float32, device=dev)
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
            self.shard_grad = torch.zeros_like(self.master_w)
            del w_full
        self.m_w, self.v_w = torch.zeros_like(self.master_w), torch.zeros_like(self.master_w)

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
        self.WT = [torch.empty(w.shape[1], w.shape[0], dtype=torch.bfloat16, device=dev) for w in self.W]
        self._refresh_transposes()

        # ---- activations (both layouts) and gradient scratch
        B, D = self.B, self.D
        self.a = [None] + [torch.empty(B, D, dtype=torch.bfloat16, device=dev) for _ in range(self.L)]
        self.aT = [None] + [torch.empty(D, B, dtype=torch.bfloat16, device=dev) for _ in range(self.L)]
        self.g = [torch.empty(B, D, dtype=torch.bfloat16, device=dev) for _ in range(2)]
        self.gT = [torch.empty(D, B, dtype=torch.bfloat16, device=dev) for _ in range(2)]
        self.dz = torch.empty(B, dtype=torch.float32, device=dev)
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=dev)

        # ---- synthetic data (different stream per rank: weak-scaling data parallelism)
        n = B * n_batches
        x, y = synthetic_batch_data(n, self.Din, seed + self.rank)
        self.X = x.to(dev, torch.bfloat16)
        self.XT = torch.empty(self.Din, n, dtype=torch.bfloat16, device=dev)
        transpose_bf16(self.X, self.XT)
        self.Y = y.to(dev)
        self.n_batches = n_batches
        kind = "allreduce" if self.zero_stage == 0 else "reducescatter+allgather"
        self.exchange = f"{comm.backend_name()}-{kind}-per-layer" if self.world_size > 1 else "none"

    # ------------------------------------------------------------------ helpers
    def _refresh_transposes(self):
        for w, wt in zip(self.W, self.WT):
            transpose_bf16(w, wt)

    def flops_per_step(self) -> int:
        return self.model.flops_per_sample() * self.B

    def grad_of(self, name: str) -> torch.Tensor:
        """This rank's local (pre-reduction) gradient of a model parameter, in its shape."""
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
        if self.world_size == 1:
            return
        bucket = self.grads_w[self.w_off[i]:self.w_off[i] + self.w_len[i]]
        if self.zero_stage == 0:
            self._collective(dist.all_reduce, bucket, works=works)
        else:
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

    # ------------------------------------------------------------------ one step
    def step(self, s: int) -> None:
        B = self.B
        j = s % self.n_batches
        x = self.X[j * B:(j + 1) * B]
        xT = self.XT[:, j * B:(j + 1) * B]
        y = self.Y[j * B:(j + 1) * B]
        # forward
        prev = x
        for i in range(self.L):
            gemm_nt(prev, self.W[i], C=self.a[i + 1], CT=self.aT[i + 1], bias=self.b[i], relu=True)
            prev = self.a[i + 1]
        # head (+ its gradients); head grads accumulate -> zero them first
        self.ghw.zero_()
        self.ghb.zero_()
        cur = 0
        mlp_head(self.a[self.L], self.hw, self.hb, y, self.dz, self.ghw, self.ghb, self.loss_acc, self.g[cur],
                 self.gT[cur])
        works: list = []
        # backward, last layer first; each weight bucket leaves as soon as its wgrad is enqueued
        for i in reversed(range(self.L)):
            a_prevT = xT if i == 0 else self.aT[i]
            gemm_nt(self.gT[cur], a_prevT, C=self.gW[i], out_f32=True)
            rowsum_bf16(self.gT[cur], self.gb[i])
            self._reduce_layer(i, works)
            if i > 0:
                gemm_nt(self.g[cur], self.WT[i], C=self.g[cur ^ 1], CT=self.gT[cur ^ 1], mask=self.a[i])
                cur ^= 1
        if self.world_size > 1:  # biases + head: one small replicated bucket
            self._collective(dist.all_reduce, self.grads_s, works=works)
        for w in works:
            w.wait()
        self.global_steps += 1
        scale = 1.0 / self.world_size
        grads_w = self.grads_w if self.zero_stage == 0 else self.shard_grad
        adam_flat_(self.master_w, grads_w, self.m_w, self.v_w, self.global_steps, self.lr, self.betas[0],
                   self.betas[1], self.eps, self.weight_decay, False, grad_scale=scale, param_lp=self.lp_w)
        adam_flat_(self.master_s, self.grads_s, self.m_s, self.v_s, self.global_steps, self.lr, self.betas[0],
                   self.betas[1], self.eps, self.weight_decay, False, grad_scale=scale)
        if self.zero_stage == 1:
            self._allgather_params()
        self._refresh_transposes()

    # bench.py adapter (same surface as TinyMLPTrainer)
    def epoch_plan(self, epoch: int):
        plan = torch.arange(self.n_batches, dtype=torch.int32).view(-1, 1)
        return plan, torch.ones(self.n_batches, dtype=torch.int32)

    def run_plan(self, plan, counts) -> None:
        for _ in range(int(plan.shape[0])):
            self.step(self.global_steps)

    @property
    def params(self) -> torch.Tensor:
        """Every parameter as this rank sees it (bf16 matrices + fp32 small params), for checks."""
        return torch.cat([self.params_bf16.float(), self.master_s])

    def check(self) -> None:
        pass

    def close(self) -> None:
        pass
