#!/usr/bin/env python3
"""Run one gemm_nt shape a few times (a compact target for rocprofv3 counter collection).

    python scripts/gemm_one.py M N K [variant] [iters] [plain|fwd]

fwd: the MLP forward's fused epilogue (bias + ReLU + C^T); hipBLASLt always runs the plain product.

variant -1 runs torch.matmul(A, B^T) (hipBLASLt) on the same operands, for side-by-side counters.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import gemm_nt  # noqa: E402

M, N, K = (int(a) for a in sys.argv[1:4])
variant = int(sys.argv[4]) if len(sys.argv) > 4 else 0
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 10
A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
fwd = len(sys.argv) > 6 and sys.argv[6] == "fwd"
CT = torch.empty(N, M, device="cuda", dtype=torch.bfloat16) if fwd else None
bias = torch.randn(N, device="cuda") if fwd else None
for _ in range(iters):
    if variant < 0:
        torch.matmul(A, B.t(), out=C)
    else:
        gemm_nt(A, B, C=C, CT=CT, bias=bias, relu=fwd, variant=variant)
torch.cuda.synchronize()
print("ok", M, N, K, variant)
