#!/usr/bin/env python3
"""The bf16 MLP's weight-gradient product dW[4096, 4096] = g^T[4096, 1024] . a^T[4096, 1024]^T
(K = batch = 1024) on every kernel that runs it -- bf16 out, and the fused wgrad + Adam epilogue --
hot and with caches flushed, against torch.matmul (hipBLASLt).  One JSON line per arm."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import gemm_nt, gemm_nt_adam_  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import bench, bench_cold  # noqa: E402

D, B = 4096, 1024
gT = torch.randn(D, B, device="cuda").bfloat16()
aT = torch.randn(D, B, device="cuda").bfloat16()
C = torch.empty(D, D, device="cuda", dtype=torch.bfloat16)
p = torch.randn(D, D, device="cuda")
m, v = torch.zeros_like(p), torch.zeros_like(p)
lp = torch.empty(D, D, device="cuda", dtype=torch.bfloat16)
arms = {}
for var in [int(x) for x in os.environ.get("VARIANTS", "0,2,9").split(",")]:
    arms[f"wgrad bf16 v{var}"] = lambda var=var: gemm_nt(gT, aT, C=C, variant=var)
    if var in (0, 2, 4, 7, 8, 9):
        arms[f"wgrad+Adam v{var}"] = lambda var=var: gemm_nt_adam_(gT, aT, p, m, v, lp, 5, 1e-4, 0.9, 0.999, 1e-8,
                                                                    variant=var)
arms["hipBLASLt gT @ aT^T"] = lambda: torch.matmul(gT, aT.t(), out=C)
for name, fn in arms.items():
    hot = bench(fn, iters=40, warmup=10)
    cold = bench_cold(fn, iters=10)
    print(json.dumps({"arm": name, "hot_us": round(hot * 1e6, 1), "cold_us": round(cold * 1e6, 1),
                      "hot_TFLOPs": round(2 * D * D * B / hot / 1e12, 1)}), flush=True)
