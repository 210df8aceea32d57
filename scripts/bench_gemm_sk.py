#!/usr/bin/env python3
"""The bf16 MLP's M = 1024 products on the split-K 256x128 kernel (variant 9) against the unsplit
128x128 kernels the shape rule ran before (forward: variant 3, front-loaded reads; [K, N] dgrad:
variant 5, software-pipelined reads) and torch.matmul (hipBLASLt, no epilogue), hot and with caches
flushed.  First a check line per product: split-K vs unsplit (max relative difference, fraction of
differing bf16 outputs).  DGT_GEMM_SK_XS picks the split-K block placement (1: a tile's K halves on
neighbouring XCDs, 0: on one XCD).  One JSON line per arm."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import gemm_nt  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import bench, bench_cold  # noqa: E402

M, N, K = 1024, 4096, 4096
xs = os.environ.get("DGT_GEMM_SK_XS", "1")
a = torch.randn(M, K, device="cuda").bfloat16()
w = torch.randn(N, K, device="cuda").bfloat16()
g = torch.randn(M, N, device="cuda").bfloat16()
C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
CT = torch.empty(N, M, device="cuda", dtype=torch.bfloat16)
bias = torch.randn(N, device="cuda")
mask = (torch.randn(M, N, device="cuda") > 0).bfloat16()
cs = torch.empty(M // 128, N, device="cuda")
prods = {
    "fwd bias+relu+T": (lambda v: gemm_nt(a, w, C=C, CT=CT, bias=bias, relu=True, variant=v), 3),
    "fwd bias+relu": (lambda v: gemm_nt(a, w, C=C, bias=bias, relu=True, variant=v), 3),
    "dgrad [K,N] mask+T+colsum": (lambda v: gemm_nt(g, w, C=C, CT=CT, mask=mask, b_kn=True, variant=v, colsum=cs), 5),
}
for name, (fn, base) in prods.items():
    fn(base)
    ref = C.float().clone()
    fn(9)
    got = C.float()
    d = (got - ref).abs()
    print(json.dumps({"check": name, "xs": xs, "max_rel_vs_unsplit": float((d / ref.abs().clamp_min(1.0)).max()),
                      "frac_differing": float((d > 0).float().mean())}), flush=True)
arms = {}
for name, (fn, base) in prods.items():
    arms[f"{name} v{base}"] = lambda fn=fn, base=base: fn(base)
    arms[f"{name} v9 xs{xs}"] = lambda fn=fn: fn(9)
arms["hipBLASLt a @ W^T"] = lambda: torch.matmul(a, w.t(), out=C)
arms["hipBLASLt g @ W"] = lambda: torch.matmul(g, w, out=C)
for name, fn in arms.items():
    hot = bench(fn, iters=40, warmup=10)
    cold = bench_cold(fn, iters=10)
    print(json.dumps({"arm": name, "hot_us": round(hot * 1e6, 1), "cold_us": round(cold * 1e6, 1),
                      "hot_TFLOPs": round(2 * M * N * K / hot / 1e12, 1)}), flush=True)
