"""Which hipBLASLt kernels torch picks for the bf16 MLP's GEMM shapes (run under rocprofv3 to read
the kernel names: macro tile MT, split GSU, stream-K SK).  Reference point for csrc/gemm.hip."""
import torch
M, D = 1024, 4096
a = torch.randn(M, D, device="cuda").bfloat16()
w = torch.randn(D, D, device="cuda").bfloat16()
g = torch.randn(M, D, device="cuda").bfloat16()
for _ in range(20):
    y = a @ w.t()          # forward  [1024, 4096] = a . W^T
    dx = g @ w             # dgrad    [1024, 4096] = g . W
    dw = g.t() @ a         # wgrad    [4096, 4096] = g^T . a
torch.cuda.synchronize()
