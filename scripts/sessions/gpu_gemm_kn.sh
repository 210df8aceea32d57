#!/bin/bash
# [K, N]-operand GEMM: correctness tests + timing vs the NT kernel on the dgrad shape.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_mlp_gemm.py -x -q -m gpu -k "b_kn" --timeout 120 --timeout-method thread > gpurun_out/pytest_kn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_kn.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_kn.log | head -20; exit $rc; }
timeout -k 10 120 python - <<'PY'
import torch, time
from distributed_gpu_test_amd.ops.gemm import gemm_nt
M, N, K = 1024, 4096, 4096
g = torch.randn(M, K, device="cuda").to(torch.bfloat16)
W = torch.randn(K, N, device="cuda").to(torch.bfloat16)   # W[out, in]
WT = W.t().contiguous()
mask = (torch.randn(M, N, device="cuda") > 0).to(torch.bfloat16)
C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda"); CT = torch.empty(N, M, dtype=torch.bfloat16, device="cuda")
flush = torch.empty(512 * 1024 * 1024 // 4, device="cuda")
for name, fn in [("nt(W^T)", lambda: gemm_nt(g, WT, C=C, CT=CT, mask=mask)), ("kn(W)", lambda: gemm_nt(g, W, C=C, CT=CT, mask=mask, b_kn=True))]:
    ts = []
    for it in range(30):
        flush.zero_(); torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e) * 1e3)
    ts = sorted(ts[5:])
    print(name, "median us", round(ts[len(ts)//2], 1), "min", round(ts[0], 1), "TF", round(2*M*N*K/ts[len(ts)//2]/1e6, 1))
ref = (g.float() @ W.float()) * (mask.float() > 0)
gemm_nt(g, W, C=C, CT=CT, mask=mask, b_kn=True); torch.cuda.synchronize()
print("max err", (C.float() - ref).abs().max().item(), "ref max", ref.abs().max().item())
PY
