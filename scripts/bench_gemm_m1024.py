#!/usr/bin/env python3
"""The bf16 MLP's M = 1024 products (forward a . W^T with bias + ReLU + C^T, dgrad g . W with the
ReLU mask + C^T, W given as [K, N]) on every kernel that can run them, hot and with caches flushed,
against torch.matmul (hipBLASLt, no epilogue).  Random N(0,1) data.  One JSON line per arm."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import gemm_nt  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import bench, bench_cold  # noqa: E402

M, N, K = 1024, 4096, 4096
a = torch.randn(M, K, device="cuda").bfloat16()
w = torch.randn(N, K, device="cuda").bfloat16()
g = torch.randn(M, N, device="cuda").bfloat16()
C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
CT = torch.empty(N, M, device="cuda", dtype=torch.bfloat16)
bias = torch.randn(N, device="cuda")
mask = (torch.randn(M, N, device="cuda") > 0).bfloat16()
# the MLP's weight gradient: dW[4096, 4096] = g^T . a over the batch (K = 1024), both operands K-major
gT = torch.randn(N, M, device="cuda").bfloat16()
aT = torch.randn(K, M, device="cuda").bfloat16()
dW = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
# variant 3 (front-loaded fragment reads) must give variant 4's bits: same MFMAs in the same order
ref, got = torch.empty_like(C), torch.empty_like(C)
gemm_nt(a, w, C=ref, CT=CT, bias=bias, relu=True, variant=4)
gemm_nt(a, w, C=got, CT=CT, bias=bias, relu=True, variant=int(os.environ.get("CHECK_VARIANT", "3")))
print(json.dumps({"check": "v%s == v4 (fwd bias+relu+T)" % os.environ.get("CHECK_VARIANT", "3"),
                  "bitwise_equal": bool(torch.equal(ref, got)),
                  "max_abs_vs_fp32": float((got.float() - torch.relu(a.float() @ w.float().t() + bias)).abs().max())}),
      flush=True)
arms = {}
for v in [int(x) for x in os.environ.get("VARIANTS", "1,4").split(",")]:
    arms[f"fwd plain v{v}"] = lambda v=v: gemm_nt(a, w, C=C, variant=v)
    arms[f"fwd bias+relu+T v{v}"] = lambda v=v: gemm_nt(a, w, C=C, CT=CT, bias=bias, relu=True, variant=v)
    arms[f"dgrad [K,N] mask+T v{v}"] = lambda v=v: gemm_nt(g, w, C=C, CT=CT, mask=mask, b_kn=True, variant=v)
for v in [int(x) for x in os.environ.get("WGRAD_VARIANTS", "").split(",") if x]:
    arms[f"wgrad 4096x4096x1024 v{v}"] = lambda v=v: gemm_nt(gT, aT, C=dW, variant=v)
if os.environ.get("WGRAD_VARIANTS"):
    arms["hipBLASLt g^T @ a (wgrad)"] = lambda: torch.matmul(gT, aT.t(), out=dW)
arms["hipBLASLt a @ W^T"] = lambda: torch.matmul(a, w.t(), out=C)
arms["hipBLASLt g @ W"] = lambda: torch.matmul(g, w, out=C)
for name, fn in arms.items():
    hot = bench(fn, iters=40, warmup=10)
    cold = bench_cold(fn, iters=10)
    print(json.dumps({"arm": name, "hot_us": round(hot * 1e6, 1), "cold_us": round(cold * 1e6, 1),
                      "hot_TFLOPs": round(2 * M * N * K / hot / 1e12, 1)}), flush=True)
