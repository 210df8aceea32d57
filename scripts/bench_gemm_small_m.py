#!/usr/bin/env python3
"""bf16 products with a small batch (M = 128 .. 1024) on 4096-wide layers: the shape rule's kernel
(variant 0; forward with bias + ReLU + C^T, [K, N] dgrad with the ReLU mask + C^T) against
torch.matmul (hipBLASLt, plain product), hot.  Below M = 1024 the 128 x 128 grid no longer fills
the chip (M = 256: 64 blocks for 256 CUs).  One JSON line per (M, product)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import gemm_nt  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import bench  # noqa: E402

N = K = 4096
variant = int(os.environ.get("VARIANT", "0"))
w = torch.randn(N, K, device="cuda").bfloat16()
bias = torch.randn(N, device="cuda")
for M in [int(m) for m in os.environ.get("MS", "128,256,512,1024").split(",")]:
    a = torch.randn(M, K, device="cuda").bfloat16()
    g = torch.randn(M, N, device="cuda").bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    CT = torch.empty(N, M, device="cuda", dtype=torch.bfloat16)
    mask = (torch.randn(M, N, device="cuda") > 0).bfloat16()
    arms = {"fwd": lambda: gemm_nt(a, w, C=C, CT=CT, bias=bias, relu=True, variant=variant),
            "dgrad": lambda: gemm_nt(g, w, C=C, CT=CT, mask=mask, b_kn=True, variant=variant),
            "blas_fwd": lambda: torch.matmul(a, w.t(), out=C),
            "blas_dgrad": lambda: torch.matmul(g, w, out=C)}
    out = {"M": M, "variant": variant}
    for k, fn in arms.items():
        out[k + "_us"] = round(bench(fn, iters=50, warmup=10) * 1e6, 1)
    print(json.dumps(out), flush=True)
