#!/usr/bin/env python3
"""The 256x256 kernel (variant 2; round 3: asm saddr DMAs, no register spills), hot, against
torch.matmul (hipBLASLt).  (The round-3 A/B arms 7 = asm DMAs and 8 = 7 + an optimizer-state
prefetch in the fused wgrad + Adam's K loop are recorded in profiles/r3_gemm256_asm_ab.jsonl; 7 is
now variant 2, 8 lost and was removed.)  Shapes: 4096^3, 8192^3, the MLP's wgrad 4096x4096x1024, and the fused wgrad + Adam
of one 4096^2 layer (state 200 MB: cold in the Infinity Cache between calls, as in the step).
One JSON line per arm."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.gemm import gemm_nt, gemm_nt_adam_  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import bench  # noqa: E402

variants = [int(x) for x in os.environ.get("VARIANTS", "2").split(",")]
reps = int(os.environ.get("REPS", "1"))
for M, N, K in [(4096, 4096, 4096), (8192, 8192, 8192), (4096, 4096, 1024)]:
    A = torch.randn(M, K, device="cuda").bfloat16()
    B = torch.randn(N, K, device="cuda").bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * M * N * K
    for r in range(reps):
        for v in variants:
            t = bench(lambda: gemm_nt(A, B, C=C, variant=v), iters=30, warmup=5)
            print(json.dumps({"shape": [M, N, K], "arm": f"v{v}", "rep": r, "us": round(t * 1e6, 1),
                              "TFLOPs": round(fl / t / 1e12, 1)}), flush=True)
    t = bench(lambda: torch.matmul(A, B.t(), out=C), iters=30, warmup=5)
    print(json.dumps({"shape": [M, N, K], "arm": "hipBLASLt", "us": round(t * 1e6, 1), "TFLOPs": round(fl / t / 1e12, 1)}), flush=True)
    del A, B, C

# fused wgrad + Adam of a 4096^2 layer: 4 layers' state rotated so each call's state is not the
# previous call's (the step's situation: 4 x 200 MB of state vs a 256 MB Infinity Cache)
D, Bt = 4096, 1024
gT = (torch.randn(D, Bt, device="cuda") * 0.1).bfloat16()
aT = (torch.randn(D, Bt, device="cuda") * 0.1).bfloat16()
layers = [[torch.randn(D, D, device="cuda"), torch.zeros(D, D, device="cuda"), torch.zeros(D, D, device="cuda"),
           torch.empty(D, D, device="cuda", dtype=torch.bfloat16)] for _ in range(4)]
for v in variants:
    st = [0]

    def run():
        L = layers[st[0] % 4]
        st[0] += 1
        gemm_nt_adam_(gT, aT, L[0], L[1], L[2], L[3], 5, 1e-4, 0.9, 0.999, 1e-8, variant=v)
    t = bench(run, iters=40, warmup=8)
    print(json.dumps({"shape": [D, D, Bt], "arm": f"wgrad+Adam v{v}", "us": round(t * 1e6, 1)}), flush=True)
