"""bf16 trainer for the bench-size synthetic MLP on the HIP MFMA GEMM (``csrc/gemm.hip``).

Reference: the loop of ``train.py:98-117`` on a bench-size ``SimpleNet`` (``train.py:26-36``).

One optimizer step, all on the GPU, no host sync:

    forward   a_l = relu(a_{l-1} W_l^T + b_l)   gemm_nt epilogue: bias + ReLU + bf16 a_l and a_l^T
    head      z = a_L w + b, BCE, dz, g_L = dz w^T * 1[a_L > 0] (+ g_L^T), dw, db      (mlp_head)
    backward  dW_l = g_l^T a_{l-1}   -> fp32 gradient buffer                           (gemm_nt)
              db_l = row sums of g_l^T                                              (rowsum_bf16)
              g_{l-1} = (g_l W_l) * 1[a_{l-1} > 0] (+ g_{l-1}^T)   epilogue: mask      (gemm_nt)
              each layer's gradient slice is all-reduced (RCCL over xGMI) as soon as its
              wgrad is enqueued: the collective overlaps the remaining backward GEMMs
    update    one fused Adam launch over the flat fp32 master (1/world_size folded in) that also
              writes the bf16 compute copy; W_l^T refreshed by a tiled transpose

Parameters live in one flat fp32 buffer (+ a bf16 mirror); per-layer segments are 64-element
aligned, so every GEMM operand and every gradient bucket is a contiguous, 16-byte aligned view.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

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
                 device: Optional[torch.device] = None):
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.model = model
        self.B, self.D, self.L, self.Din = batch_size, model.width, model.depth, model.in_features
        self.rank, self.world_size = comm.get_rank(), comm.get_world_size()
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.global_steps = 0
        dev = self.device

        # ---- flat parameter layout: [W_l, b_l]*, head.w, head.b
        self.segments: List[Tuple[str, Tuple[int, ...], int]] = []
        off = 0
        for name, p in model.named_parameters():
            self.segments.append((name, tuple(p.shape), off))
            off = _round(off + p.numel())
        self.total = off
        master = torch.zeros(self.total, dtype=torch.float32)
        for (name, shape, o), p in zip(self.segments, model.parameters()):
            master[o:o + p.numel()] = p.detach().reshape(-1).float()
        self.master = master.to(dev)
        comm.broadcast_(self.master, 0)
        self.params_bf16 = self.master.to(torch.bfloat16)
        self.grads = torch.zeros_like(self.master)
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        seg = {n: (s, o) for n, s, o in self.segments}

        def view(buf, name):
            shape, o = seg[name]
            n = 1
            for d in shape:
                n *= d
            return buf[o:o + n].view(shape)

        self.W = [view(self.params_bf16, f"layers.{i}.weight") for i in range(self.L)]
        self.b = [view(self.master, f"layers.{i}.bias") for i in range(self.L)]
        self.gW = [view(self.grads, f"layers.{i}.weight") for i in range(self.L)]
        self.gb = [view(self.grads, f"layers.{i}.bias") for i in range(self.L)]
        self.hw = view(self.master, "head.weight").view(-1)
        self.hb = view(self.master, "head.bias").view(-1)
        self.ghw = view(self.grads, "head.weight").view(-1)
        self.ghb = view(self.grads, "head.bias").view(-1)
        self.layer_slices = []  # contiguous gradient bucket per layer (W_l, b_l)
        for i in range(self.L):
            _, o_w = seg[f"layers.{i}.weight"]
            shape_b, o_b = seg[f"layers.{i}.bias"]
            self.layer_slices.append((o_w, _round(o_b + shape_b[0])))
        _, o_h = seg["head.weight"]
        self.layer_slices.append((o_h, self.total))
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
        self.exchange = f"{comm.backend_name()}-allreduce-per-layer" if self.world_size > 1 else "none"

    # ------------------------------------------------------------------ helpers
    def _refresh_transposes(self):
        for w, wt in zip(self.W, self.WT):
            transpose_bf16(w, wt)

    def flops_per_step(self) -> int:
        return self.model.flops_per_sample() * self.B

    def _reduce_async(self, li: int, works: list):
        if self.world_size == 1:
            return
        lo, hi = self.layer_slices[li]
        view = self.grads[lo:hi]
        if comm.needs_host_staging(view):
            comm.all_reduce_(view)
        else:
            works.append(dist.all_reduce(view, async_op=True))

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
        self._reduce_async(self.L, works)
        # backward, last layer first; each layer's gradient bucket leaves as soon as it is enqueued
        for i in reversed(range(self.L)):
            a_prevT = xT if i == 0 else self.aT[i]
            gemm_nt(self.gT[cur], a_prevT, C=self.gW[i], out_f32=True)
            rowsum_bf16(self.gT[cur], self.gb[i])
            self._reduce_async(i, works)
            if i > 0:
                gemm_nt(self.g[cur], self.WT[i], C=self.g[cur ^ 1], CT=self.gT[cur ^ 1], mask=self.a[i])
                cur ^= 1
        for w in works:
            w.wait()
        self.global_steps += 1
        adam_flat_(self.master, self.grads, self.exp_avg, self.exp_avg_sq, self.global_steps, self.lr,
                   self.betas[0], self.betas[1], self.eps, self.weight_decay, False,
                   grad_scale=1.0 / self.world_size, param_lp=self.params_bf16)
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
        return self.master

    def check(self) -> None:
        pass

    def close(self) -> None:
        pass
