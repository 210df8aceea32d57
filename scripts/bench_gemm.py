#!/usr/bin/env python3
"""GEMM micro-benchmark: the HIP MFMA gemm_nt kernel vs torch.matmul (hipBLASLt) on the MLP's
shapes, bf16 in / fp32 accumulate, random N(0,1) data (cdna_hip_programming.md rule 25).
Prints one JSON line per shape."""
import json
import sys
import os
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import gemm_nt  # noqa: E402


def bench(fn, iters=50, warmup=10):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


_FLUSH = None


def bench_cold(fn, iters=10):
    """Per-call time with L2 and the 256 MB Infinity Cache flushed before every call (a 1 GiB write),
    the situation inside a training step where the optimizer streams GBs between GEMMs."""
    global _FLUSH
    if _FLUSH is None:
        _FLUSH = torch.empty(1 << 28, device="cuda")
    total = 0.0
    for _ in range(iters + 2):
        _FLUSH.fill_(1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        total += e0.elapsed_time(e1) * 1e-3 if _ >= 2 else 0.0
    return total / iters


def main():
    shapes = [(4096, 4096, 4096), (8192, 8192, 8192), (1024, 4096, 4096), (4096, 4096, 1024), (2048, 8192, 8192)]
    for M, N, K in shapes:
        A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        Cf = torch.empty(M, N, device="cuda", dtype=torch.float32)
        flops = 2.0 * M * N * K
        t_ours = bench(lambda: gemm_nt(A, B, C=C))
        t_ours32 = bench(lambda: gemm_nt(A, B, C=Cf, out_f32=True))
        t_128 = bench(lambda: gemm_nt(A, B, C=C, variant=1))
        t_128d = None
        t_128e = bench(lambda: gemm_nt(A, B, C=C, variant=4))
        fits256 = M % 256 == 0 and N % 256 == 0 and K % 128 == 0
        t_256 = bench(lambda: gemm_nt(A, B, C=C, variant=2)) if fits256 else None
        t_torch = bench(lambda: torch.matmul(A, B.t(), out=C))
        extra = {}
        if M == 1024:  # the MLP's forward / dgrad shapes with their fused epilogues
            bias = torch.randn(N, device="cuda")
            CT = torch.empty(N, M, device="cuda", dtype=torch.bfloat16)
            mask = (torch.randn(M, N, device="cuda") > 0).to(torch.bfloat16)
            extra["fwd_bias_relu_T_us"] = round(bench(lambda: gemm_nt(A, B, C=C, CT=CT, bias=bias, relu=True)) * 1e6, 1)
            extra["fwd_bias_relu_us"] = round(bench(lambda: gemm_nt(A, B, C=C, bias=bias, relu=True)) * 1e6, 1)
            extra["T_only_us"] = round(bench(lambda: gemm_nt(A, B, CT=CT, bias=bias, relu=True)) * 1e6, 1)
            extra["dgrad_mask_T_us"] = round(bench(lambda: gemm_nt(A, B, C=C, CT=CT, mask=mask)) * 1e6, 1)
            extra["fwd_bias_relu_T_cold_us"] = round(bench_cold(lambda: gemm_nt(A, B, C=C, CT=CT, bias=bias, relu=True)) * 1e6, 1)
            extra["fwd_bias_relu_T_cold_8wave_us"] = round(bench_cold(lambda: gemm_nt(A, B, C=C, CT=CT, bias=bias, relu=True, variant=4)) * 1e6, 1)
            extra["fwd_bias_relu_T_cold_2stage_us"] = round(bench_cold(lambda: gemm_nt(A, B, C=C, CT=CT, bias=bias, relu=True, variant=1)) * 1e6, 1)
            extra["torch_cold_us"] = round(bench_cold(lambda: torch.matmul(A, B.t(), out=C)) * 1e6, 1)
        print(json.dumps({"M": M, "N": N, "K": K, "dgt_TFLOPs": round(flops / t_ours / 1e12, 1),
                          "dgt_f32out_TFLOPs": round(flops / t_ours32 / 1e12, 1),
                          "dgt_tile128_TFLOPs": round(flops / t_128 / 1e12, 1),
                          "dgt_tile128_4stage_TFLOPs": round(flops / t_128d / 1e12, 1),
                          "dgt_tile128_4stage_8wave_TFLOPs": round(flops / t_128e / 1e12, 1),
                          "dgt_tile256_TFLOPs": round(flops / t_256 / 1e12, 1) if t_256 else None,
                          "torch_hipblaslt_TFLOPs": round(flops / t_torch / 1e12, 1),
                          "dgt_us": round(t_ours * 1e6, 1), "torch_us": round(t_torch * 1e6, 1), **extra}), flush=True)


if __name__ == "__main__":
    main()
