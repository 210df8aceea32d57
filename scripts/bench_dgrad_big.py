#!/usr/bin/env python3
"""The [K, N] dgrad (g . W with the ReLU mask + C^T) on grids larger than the chip (batch 2048 / 4096
on 4096- and 8192-wide layers): the shape rule's 2-stage 128x128 kernel (v0 / v1) against the
8-wave kernels forced (v3 front-loaded reads, v4 plain, v5 software-pipelined) and hipBLASLt, hot."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import gemm_nt  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import bench  # noqa: E402

for M, W in [(2048, 4096), (4096, 4096), (2048, 8192)]:
    g = torch.randn(M, W, device="cuda").bfloat16()
    w = torch.randn(W, W, device="cuda").bfloat16()
    C = torch.empty(M, W, device="cuda", dtype=torch.bfloat16)
    CT = torch.empty(W, M, device="cuda", dtype=torch.bfloat16)
    mask = (torch.randn(M, W, device="cuda") > 0).bfloat16()
    cs = torch.empty(M // 128, W, device="cuda")
    fl = 2.0 * M * W * W
    out = {"M": M, "W": W}
    for v in (0, 1, 3, 4, 5):
        out[f"v{v}_us"] = round(bench(lambda v=v: gemm_nt(g, w, C=C, CT=CT, mask=mask, b_kn=True, colsum=cs, variant=v),
                                      iters=20, warmup=5) * 1e6, 1)
    out["blas_us"] = round(bench(lambda: torch.matmul(g, w, out=C), iters=20, warmup=5) * 1e6, 1)
    print(json.dumps(out), flush=True)
