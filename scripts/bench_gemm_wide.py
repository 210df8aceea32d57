#!/usr/bin/env python3
"""bf16 products of an 8192-wide MLP layer (F = H = 4096-8192) at batch 1024 / 2048:
forward (bias + ReLU + C^T), [K, N] dgrad (mask + C^T), wgrad (bf16 out) on the shape rule's kernel
(variant 0) and on each tile family, against torch.matmul (hipBLASLt), hot.  One JSON line each."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import gemm_nt  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import bench  # noqa: E402

W = int(os.environ.get("WIDTH", "8192"))
for M in [int(m) for m in os.environ.get("MS", "1024,2048").split(",")]:
    a = torch.randn(M, W, device="cuda").bfloat16()
    w = torch.randn(W, W, device="cuda").bfloat16()
    g = torch.randn(M, W, device="cuda").bfloat16()
    gT, aT = g.t().contiguous(), a.t().contiguous()
    C = torch.empty(M, W, device="cuda", dtype=torch.bfloat16)
    CT = torch.empty(W, M, device="cuda", dtype=torch.bfloat16)
    dW = torch.empty(W, W, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(W, device="cuda")
    mask = (torch.randn(M, W, device="cuda") > 0).bfloat16()
    fl = 2.0 * M * W * W
    arms = {}
    for v in (0, 3, 8):
        arms[f"fwd v{v}"] = lambda v=v: gemm_nt(a, w, C=C, CT=CT, bias=bias, relu=True, variant=v)
        arms[f"wgrad v{v}"] = lambda v=v: gemm_nt(gT, aT, C=dW, variant=v)
    for v in (0, 3):
        arms[f"dgrad v{v}"] = lambda v=v: gemm_nt(g, w, C=C, CT=CT, mask=mask, b_kn=True, variant=v)
    arms["blas fwd"] = lambda: torch.matmul(a, w.t(), out=C)
    arms["blas dgrad"] = lambda: torch.matmul(g, w, out=C)
    arms["blas wgrad"] = lambda: torch.matmul(gT, aT.t(), out=dW)
    for k, fn in arms.items():
        try:
            us = bench(fn, iters=20, warmup=5) * 1e6
            print(json.dumps({"M": M, "width": W, "arm": k, "us": round(us, 1), "PF": round(fl / us / 1e9, 3)}), flush=True)
        except RuntimeError as e:
            print(json.dumps({"M": M, "width": W, "arm": k, "error": str(e)[:100]}), flush=True)
