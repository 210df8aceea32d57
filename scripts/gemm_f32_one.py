#!/usr/bin/env python3
"""One exact-fp32 Linear product a few times (a compact rocprofv3 counter target).

    python scripts/gemm_f32_one.py M N K [fwd|dgrad|wgrad|blas] [iters]

blas runs torch.mm (hipBLASLt fp32) on the forward's operands."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops import _ext  # noqa: E402

M, N, K = (int(a) for a in sys.argv[1:4])
prod = sys.argv[4] if len(sys.argv) > 4 else "fwd"
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 10
ops = _ext.require()
x, W = torch.randn(M, K, device="cuda"), torch.randn(N, K, device="cuda")
dy, y = torch.randn(M, N, device="cuda"), torch.empty(M, N, device="cuda")
dx, dW = torch.empty(M, K, device="cuda"), torch.empty(N, K, device="cuda")
for _ in range(iters):
    if prod == "fwd":
        ops.gemm_f32(x, W, None, None, y, 0, 0, False, False)
    elif prod == "dgrad":
        ops.gemm_f32(dy, W, None, None, dx, 0, 1, False, False)
    elif prod == "wgrad":
        ops.gemm_f32(dy, x, None, None, dW, 1, 1, False, False)
    else:
        torch.mm(x, W.t(), out=y)
torch.cuda.synchronize()
print("ok", M, N, K, prod)
