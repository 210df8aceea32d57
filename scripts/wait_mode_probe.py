"""Launch -> completion -> host wake-up round trip under the HIP runtime's wait modes.

    DGT_HIP_SPIN=1   hipSetDeviceFlags(hipDeviceScheduleSpin) before torch creates the context
    ROC_ACTIVE_WAIT_TIMEOUT=<us>  (runtime env) how long a blocking wait spins before sleeping

Prints us per (one-element add_ + synchronize) and per (fused tiny-MLP launch of K steps + synchronize)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("DGT_HIP_SPIN") == "1":
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipSetDevice(0) == 0
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
    print(f"hipSetDeviceFlags(spin) rc={rc}", flush=True)
import torch  # noqa: E402

import bench  # noqa: E402
from distributed_gpu_test_amd.data import make_synthetic_data  # noqa: E402
from distributed_gpu_test_amd.models import SimpleNet  # noqa: E402
from distributed_gpu_test_amd.runtime.tiny_trainer import TinyMLPTrainer  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(42)
x, y = make_synthetic_data(2000, 20, 42)
tr = TinyMLPTrainer(SimpleNet(20, 64), x, y, 4, impl="fused", device=dev)
plan, counts = bench.build_plan(tr, 100000)


def t(label, f, n=500):
    for _ in range(50):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"{label:36s} median {ts[n // 2] * 1e6:7.2f} us  p10 {ts[n // 10] * 1e6:7.2f}  p90 {ts[9 * n // 10] * 1e6:7.2f}",
          flush=True)


z = torch.zeros(1, device=dev)


def add_sync():
    z.add_(1)
    torch.cuda.synchronize()


t("add_ + synchronize", add_sync)
for K in (1, 20):
    p, c = plan[:K].contiguous(), counts[:K].contiguous()

    def run(p=p, c=c):
        tr.run_plan(p, c)
        torch.cuda.synchronize()
    t(f"fused K={K} + synchronize", run)
