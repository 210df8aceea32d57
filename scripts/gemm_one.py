#!/usr/bin/env python3
"""Run one gemm_nt shape a few times (a compact target for rocprofv3 counter collection).

    python scripts/gemm_one.py M N K [variant] [iters] [plain|fwd]

fwd: the MLP forward's fused epilogue (bias + ReLU + C^T); hipBLASLt always runs the plain product.
dgrad: the MLP dgrad -- B given as [K, N] (W as it lies), ReLU mask + C^T + bias-gradient column
sums; variant -1 then runs torch.matmul(A, B) on the same [K, N] operand.

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
mode = sys.argv[6] if len(sys.argv) > 6 else "plain"
fwd, dgrad = mode == "fwd", mode == "dgrad"
A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
B = torch.randn(*((K, N) if dgrad else (N, K)), device="cuda").to(torch.bfloat16)
C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
CT = torch.empty(N, M, device="cuda", dtype=torch.bfloat16) if (fwd or dgrad) else None
bias = torch.randn(N, device="cuda") if fwd else None
mask = (torch.randn(M, N, device="cuda") > 0).to(torch.bfloat16) if dgrad else None
cs = torch.empty(M // 128, N, device="cuda") if dgrad else None
for _ in range(iters):
    if variant < 0:
        torch.matmul(A, B if dgrad else B.t(), out=C)
    elif dgrad:
        gemm_nt(A, B, C=C, CT=CT, mask=mask, b_kn=True, colsum=cs, variant=variant)
    else:
        gemm_nt(A, B, C=C, CT=CT, bias=bias, relu=fwd, variant=variant)
torch.cuda.synchronize()
print("ok", M, N, K, variant)
