#!/usr/bin/env python3
"""256 x 256 kernels (variant 2: 8-phase, variant 9: two stages, one barrier per K-tile) across
square and K = 1024 shapes, bf16 and fp32 out, hot / cold.  One JSON line per arm."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import gemm_nt  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import bench, bench_cold  # noqa: E402

for M, N, K in [(4096, 4096, 1024), (4096, 4096, 4096), (8192, 8192, 8192), (8192, 8192, 1024)]:
    A = torch.randn(M, K, device="cuda").bfloat16()
    B = torch.randn(N, K, device="cuda").bfloat16()
    for out in ("bf16", "f32"):
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16 if out == "bf16" else torch.float32)
        for v in (2, 9):
            fn = lambda v=v: gemm_nt(A, B, C=C, out_f32=out == "f32", variant=v)
            hot = bench(fn, iters=20, warmup=5)
            cold = bench_cold(fn, iters=5)
            print(json.dumps({"shape": [M, N, K], "out": out, "variant": v, "hot_us": round(hot * 1e6, 1),
                              "cold_us": round(cold * 1e6, 1), "hot_TFLOPs": round(2 * M * N * K / hot / 1e12, 1)}),
                  flush=True)
    fn = lambda: torch.matmul(A, B.t())
    hot = bench(fn, iters=20, warmup=5)
    print(json.dumps({"shape": [M, N, K], "out": "bf16", "variant": "hipBLASLt", "hot_us": round(hot * 1e6, 1),
                      "hot_TFLOPs": round(2 * M * N * K / hot / 1e12, 1)}), flush=True)
