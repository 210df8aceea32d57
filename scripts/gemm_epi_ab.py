#!/usr/bin/env python3
"""Hot time of the bf16 MLP's three M = 1024 product kinds on the shape rule's kernels (variant 0),
for A/B runs of the extension (DGT_EXT_LIB): forward with bias + ReLU + C^T, forward with bias +
ReLU, dgrad from W as [K, N] with ReLU mask + C^T + bias-gradient partials.  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import gemm_nt  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import bench  # noqa: E402

M, N, K = 1024, 4096, 4096
a = torch.randn(M, K, device="cuda").bfloat16()
w = torch.randn(N, K, device="cuda").bfloat16()
g = torch.randn(M, N, device="cuda").bfloat16()
C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
CT = torch.empty(N, M, device="cuda", dtype=torch.bfloat16)
bias = torch.randn(N, device="cuda")
mask = (torch.randn(M, N, device="cuda") > 0).bfloat16()
cs = torch.empty(M // 128, N, device="cuda")
out = {"ext": os.environ.get("DGT_EXT_LIB", "in-tree")}
for name, fn in [("fwd_T", lambda: gemm_nt(a, w, C=C, CT=CT, bias=bias, relu=True)),
                 ("fwd", lambda: gemm_nt(a, w, C=C, bias=bias, relu=True)),
                 ("dgrad", lambda: gemm_nt(g, w, C=C, CT=CT, mask=mask, b_kn=True, colsum=cs))]:
    out[name] = round(bench(fn, iters=60, warmup=10) * 1e6, 2)
print(json.dumps(out), flush=True)
