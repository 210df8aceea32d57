#!/usr/bin/env python3
"""The MLP's weight-gradient GEMM + Adam on one 4096 x 4096 layer (batch 1024, bf16), every way
this framework can run it: fused (gemm_nt_adam_, one launch, per kernel variant) against the
unfused pair (wgrad GEMM into a bf16 gradient, then the flat Adam).  Random data; prints one JSON
line per arm with the per-layer time."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.adam import adam_flat_  # noqa: E402
from distributed_gpu_test_amd.ops.gemm import gemm_nt, gemm_nt_adam_  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import bench  # noqa: E402

D, B = int(os.environ.get("D", 4096)), int(os.environ.get("B", 1024))
g = torch.Generator().manual_seed(0)
gT = (torch.randn(D, B, generator=g) * 0.1).to(torch.bfloat16).cuda()
aT = (torch.randn(D, B, generator=g) * 0.1).to(torch.bfloat16).cuda()
master = torch.randn(D, D, generator=g).cuda()
m, v = torch.zeros(D, D, device="cuda"), torch.zeros(D, D, device="cuda")
lp = torch.empty(D, D, dtype=torch.bfloat16, device="cuda")
grad = torch.empty(D, D, dtype=torch.bfloat16, device="cuda")
args = (1, 1e-4, 0.9, 0.999, 1e-8, 0.0, False)


def unfused():
    gemm_nt(gT, aT, C=grad)
    adam_flat_(master.view(-1), grad.view(-1), m.view(-1), v.view(-1), *args, param_lp=lp.view(-1))


arms = {"unfused (wgrad bf16 + flat Adam)": unfused, "wgrad GEMM alone": lambda: gemm_nt(gT, aT, C=grad),
        "flat Adam alone": lambda: adam_flat_(master.view(-1), grad.view(-1), m.view(-1), v.view(-1), *args,
                                               param_lp=lp.view(-1))}
for var in (0, 1, 2, 3, 4, 6):
    arms[f"fused variant {var}"] = (lambda var=var: gemm_nt_adam_(gT, aT, master, m, v, lp, *args, variant=var))
for name, fn in arms.items():
    t = bench(fn, iters=30, warmup=5)
    print(json.dumps({"arm": name, "us": round(t * 1e6, 1), "D": D, "B": B}), flush=True)
