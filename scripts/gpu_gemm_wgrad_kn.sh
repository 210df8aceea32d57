#!/bin/bash
# wgrad dW[out,in] = g^T . a: NT(g^T, a^T) (256x256 kernel) vs KN(g^T, a) (128x128, transposed reads);
# forward with and without the C^T epilogue.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python - <<'PY'
import torch
from distributed_gpu_test_amd.ops.gemm import gemm_nt
B, D = 1024, 4096
gT = torch.randn(D, B, device="cuda").to(torch.bfloat16)
a = torch.relu(torch.randn(B, D, device="cuda")).to(torch.bfloat16)
aT = a.t().contiguous()
W = torch.randn(D, D, device="cuda").to(torch.bfloat16)
bias = torch.randn(D, device="cuda")
C = torch.empty(D, D, dtype=torch.bfloat16, device="cuda")
Ca = torch.empty(B, D, dtype=torch.bfloat16, device="cuda"); CaT = torch.empty(D, B, dtype=torch.bfloat16, device="cuda")
flush = torch.empty(512 * 1024 * 1024 // 4, device="cuda")
def t(fn):
    ts = []
    for it in range(30):
        flush.zero_(); torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e) * 1e3)
    ts = sorted(ts[5:]); return round(ts[len(ts)//2], 1)
cases = [("wgrad NT 256x256", lambda: gemm_nt(gT, aT, C=C)),
         ("wgrad KN v0", lambda: gemm_nt(gT, a, C=C, b_kn=True)),
         ("wgrad KN v1 (2-stage)", lambda: gemm_nt(gT, a, C=C, b_kn=True, variant=1)),
         ("wgrad KN v3 (4-stage)", lambda: gemm_nt(gT, a, C=C, b_kn=True, variant=3)),
         ("wgrad KN v4 (4-stage 8w)", lambda: gemm_nt(gT, a, C=C, b_kn=True, variant=4)),
         ("fwd with C^T", lambda: gemm_nt(a, W, C=Ca, CT=CaT, bias=bias, relu=True)),
         ("fwd no C^T", lambda: gemm_nt(a, W, C=Ca, bias=bias, relu=True))]
for name, fn in cases:
    print(f"{name:28s} {t(fn):8.1f} us")
ref = gT.float() @ a.float()
gemm_nt(gT, a, C=C, b_kn=True); torch.cuda.synchronize()
print("kn max rel err", ((C.float() - ref).abs().max() / ref.abs().max()).item())
PY
