#!/usr/bin/env python3
"""transpose_bf16 (csrc/gemm.hip, the register-tile kernel) vs torch .t().contiguous(), hot, GB/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import transpose_bf16  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import bench  # noqa: E402

for r, c in [(1024, 4096), (4096, 4096), (8192, 8192)]:
    x = torch.randn(r, c, device="cuda").bfloat16()
    y = torch.empty(c, r, device="cuda", dtype=torch.bfloat16)
    ours = bench(lambda: transpose_bf16(x, y), iters=50, warmup=10)
    tor = bench(lambda: y.copy_(x.t()), iters=50, warmup=10)
    assert torch.equal(y, x.t())
    gb = 2 * r * c * 2 / 1e9
    print(json.dumps({"rows": r, "cols": c, "ours_us": round(ours * 1e6, 1), "ours_TBps": round(gb / ours / 1e3, 2),
                      "torch_us": round(tor * 1e6, 1), "torch_TBps": round(gb / tor / 1e3, 2)}), flush=True)
