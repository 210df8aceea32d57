#!/usr/bin/env python3
"""Time torch.matmul (hipBLASLt) on the MLP's GEMM shapes, for comparison with csrc/gemm.hip; run
under rocprofv3 --kernel-trace to see which macro tile hipBLASLt picks.

    python scripts/hipblaslt_probe.py
"""
import torch

shapes = [(1024, 4096, 4096), (4096, 4096, 1024)]
for M, N, K in shapes:
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    for _ in range(10):
        c = a @ b.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        c = a @ b.t()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 50
    print(f"hipBLASLt M={M} N={N} K={K}: {us:.1f} us  {2 * M * N * K / us / 1e6:.0f} TF", flush=True)
