#!/bin/bash
# M=1024 GEMM shapes: hot-cache vs cold-cache (flushed) timings per variant.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 180 python - <<'PY'
import torch
from distributed_gpu_test_amd.ops.gemm import gemm_nt
M, N, K = 1024, 4096, 4096
A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
CT = torch.empty(N, M, dtype=torch.bfloat16, device="cuda")
bias = torch.randn(N, device="cuda")
flush = torch.empty(512 * 1024 * 1024 // 4, device="cuda")
def t(fn, cold):
    ts = []
    for it in range(40):
        if cold:
            flush.zero_()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e) * 1e3)
    ts = sorted(ts[5:]); return ts[len(ts)//2]
for v in (1, 4):
    for name, fn in [("plain", lambda: gemm_nt(A, B, C=C, variant=v)),
                     ("fwd epi", lambda: gemm_nt(A, B, C=C, CT=CT, bias=bias, relu=True, variant=v))]:
        print(f"variant {v} {name:8s} hot {t(fn, False):6.1f} us  cold {t(fn, True):6.1f} us")
ts = []
for it in range(40):
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(); torch.matmul(A, B.t(), out=C); e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e) * 1e3)
ts = sorted(ts[5:]); print("hipBLASLt hot", ts[len(ts)//2])
PY
