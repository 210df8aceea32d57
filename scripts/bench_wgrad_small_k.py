#!/usr/bin/env python3
"""The bf16 MLP's weight gradient at small per-GPU batch: dW[4096, 4096] = g^T . a with K = batch
(both operands K-major), bf16 out, on the shape rule's kernel (variant 0: 256x256 for >= 200 tiles),
the 128x128 kernel (variant 3) and torch.matmul (hipBLASLt), hot.  One JSON line per K."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import gemm_nt  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import bench  # noqa: E402

N = 4096
for K in [int(k) for k in os.environ.get("KS", "128,256,512,1024").split(",")]:
    gT = torch.randn(N, K, device="cuda").bfloat16()
    aT = torch.randn(N, K, device="cuda").bfloat16()
    dW = torch.empty(N, N, device="cuda", dtype=torch.bfloat16)
    out = {"K": K}
    for name, fn in [("v0", lambda: gemm_nt(gT, aT, C=dW)), ("v3", lambda: gemm_nt(gT, aT, C=dW, variant=3)),
                     ("v1", lambda: gemm_nt(gT, aT, C=dW, variant=1)),
                     ("blas", lambda: torch.matmul(gT, aT.t(), out=dW))]:
        out[name + "_us"] = round(bench(fn, iters=50, warmup=10) * 1e6, 1)
    print(json.dumps(out), flush=True)
