#!/usr/bin/env python3
"""The shape rule's 256x256 kernel (cross-phase prefetch) on M = N = 4096 over K = 128 .. 4096, hot:
a linear fit of time against K-tiles separates the fixed cost (launch, pipeline fill, epilogue)
from the per-K-tile cost.  One JSON line per K, then the fit."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import gemm_nt  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import bench  # noqa: E402

M = N = 4096
C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
pts = []
for K in (128, 256, 512, 1024, 2048, 4096):
    A = torch.randn(M, K, device="cuda").bfloat16()
    B = torch.randn(N, K, device="cuda").bfloat16()
    t = bench(lambda: gemm_nt(A, B, C=C), iters=30, warmup=5) * 1e6
    tb = bench(lambda: torch.matmul(A, B.t(), out=C), iters=30, warmup=5) * 1e6
    pts.append((K // 64, t))
    print(json.dumps({"shape": [M, N, K], "ours_us": round(t, 2), "hipBLASLt_us": round(tb, 2)}), flush=True)
n = len(pts)
sx = sum(p[0] for p in pts); sy = sum(p[1] for p in pts)
sxx = sum(p[0] ** 2 for p in pts); sxy = sum(p[0] * p[1] for p in pts)
slope = (n * sxy - sx * sy) / (n * sxx - sx * sx)
print(json.dumps({"fit": "us = fixed + per_ktile * K/64", "fixed_us": round((sy - slope * sx) / n, 2),
                  "per_ktile_us": round(slope, 3)}), flush=True)
