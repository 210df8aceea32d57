"""Probe: would split-K on the 256x256 kernel beat the 128x128 kernels at the MLP's M = 1024 shapes?

At M = 1024, N = K = 4096 the 128x128 tile grid is exactly one block per CU and each CU fetches
32 KiB from L2 per 2.1 MFLOP K-tile -- as many L2 cycles as MFMA cycles.  A 256x256 tile halves the
fetch per FLOP but gives only 64 tiles; splitting K four ways restores 256 blocks.  This times the
four K-quarter GEMMs (fp32 partial outputs, the 256x256 kernel = variant 2) launched on four streams
at once, against the current forward (128x128, bias + ReLU + C^T epilogue) and its plain product.
The partial-sum reduction + epilogue is timed as torch's sum (an upper bound for a fused kernel).
Prints one JSON line per arm.
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from distributed_gpu_test_amd.ops.gemm import gemm_nt  # noqa: E402

M, N, K, S = 1024, 4096, 4096, 4
REPS = 50
dev = torch.device("cuda")
g = torch.Generator().manual_seed(0)
A = torch.randn(M, K, generator=g).bfloat16().to(dev)
W = (torch.randn(N, K, generator=g) * 0.02).bfloat16().to(dev)
bias = torch.randn(N, generator=g).bfloat16().to(dev)
C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
CT = torch.empty(N, M, dtype=torch.bfloat16, device=dev)
P = torch.empty(S, M, N, dtype=torch.float32, device=dev)
streams = [torch.cuda.Stream() for _ in range(S)]
kq = K // S


def timed(fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / REPS


def split_concurrent():
    cur = torch.cuda.current_stream()
    for q, s in enumerate(streams):
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            gemm_nt(A[:, q * kq:(q + 1) * kq], W[:, q * kq:(q + 1) * kq], C=P[q], out_f32=True, variant=2)
    for s in streams:
        cur.wait_stream(s)


def split_serial():
    for q in range(S):
        gemm_nt(A[:, q * kq:(q + 1) * kq], W[:, q * kq:(q + 1) * kq], C=P[q], out_f32=True, variant=2)


arms = {
    "fwd 128x128 bias+relu+CT (current)": lambda: gemm_nt(A, W, C=C, CT=CT, bias=bias, relu=True),
    "fwd 128x128 plain": lambda: gemm_nt(A, W, C=C),
    "split-K 4 x 256x256 fp32, 4 streams": split_concurrent,
    "split-K 4 x 256x256 fp32, 1 stream": split_serial,
    "one K-quarter 256x256 (64 blocks)": lambda: gemm_nt(A[:, :kq], W[:, :kq], C=P[0], out_f32=True, variant=2),
    "torch reduce of the 4 partials": lambda: P.sum(0),
}
ref = (A.float() @ W.float().t())
split_concurrent()
torch.cuda.synchronize()
err = float((P.sum(0) - ref).abs().max() / ref.abs().max())
for name, fn in arms.items():
    print(json.dumps({"arm": name, "us": round(timed(fn), 2), "shape": [M, N, K]}), flush=True)
print(json.dumps({"split_rel_err_vs_fp32": err}), flush=True)
