#!/usr/bin/env python3
"""Exact-fp32 MFMA GEMM (csrc/gemm_f32.hip) vs torch.matmul (hipBLASLt fp32) on the Linear products:
forward (x W^T), dgrad (g W), wgrad (g^T x) at the engine's fp32 shapes.  Hot timing: CUDA events
around `iters` back-to-back launches after warmup; one JSON line per (shape, product)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_gpu_test_amd.ops import _ext  # noqa: E402


def timed(fn, iters=50, warm=10):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ops = _ext.require()
    shapes = [(1024, 1024, 1024), (1024, 4096, 4096), (4096, 4096, 4096), (2048, 2048, 2048), (8192, 8192, 8192),
              (256, 4096, 4096), (1000, 1000, 1000)]
    if len(sys.argv) > 1:
        shapes = [tuple(int(v) for v in s.split("x")) for s in sys.argv[1:]]
    for M, N, K in shapes:  # Linear(K -> N) on a batch of M
        x = torch.randn(M, K, device="cuda")
        W = torch.randn(N, K, device="cuda")
        b = torch.randn(N, device="cuda")
        dy = torch.randn(M, N, device="cuda")
        y = torch.empty(M, N, device="cuda")
        dx = torch.empty(M, K, device="cuda")
        dW = torch.empty(N, K, device="cuda")
        prods = {
            "fwd": (lambda: ops.gemm_f32(x, W, None, b, y, 0, 0, True, False),
                    lambda: torch.addmm(b, x, W.t()), 2 * M * N * K),
            "dgrad": (lambda: ops.gemm_f32(dy, W, None, None, dx, 0, 1, False, False),
                      lambda: torch.mm(dy, W), 2 * M * N * K),
            "wgrad": (lambda: ops.gemm_f32(dy, x, None, None, dW, 1, 1, False, False),
                      lambda: torch.mm(dy.t(), x), 2 * M * N * K),
        }
        iters = max(3, min(50, int(2e12 / (2 * M * N * K))))
        for name, (ours, theirs, flop) in prods.items():
            t_ours = timed(ours, iters)
            t_blas = timed(theirs, iters)
            print(json.dumps({"M": M, "N": N, "K": K, "product": name, "ours_us": round(t_ours, 2),
                              "hipblaslt_us": round(t_blas, 2), "ours_TF": round(flop / t_ours / 1e6, 1),
                              "hipblaslt_TF": round(flop / t_blas / 1e6, 1),
                              "speedup": round(t_blas / t_ours, 3)}), flush=True)


if __name__ == "__main__":
    main()
