"""Launch -> completion -> host wake-up round trip under a HIP device scheduling mode.

usage: python scripts/sync_mode_probe.py {auto|spin|yield|blocking}

Sets hipSetDeviceFlags on torch's own HIP runtime before anything touches the device, then times
(a) a trivial torch kernel + synchronize and (b) the fused trainer at K = 1 / 10 / 100 + synchronize.
This is the fixed cost of one timed bench run (profiles/r1_fused_launch_overhead.txt)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

FLAGS = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}
mode = sys.argv[1] if len(sys.argv) > 1 else "auto"
hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
rc = hip.hipSetDeviceFlags(ctypes.c_uint(FLAGS[mode]))
flags = ctypes.c_uint(0)
hip.hipGetDeviceFlags(ctypes.byref(flags))
print(f"mode={mode} hipSetDeviceFlags rc={rc} flags=0x{flags.value:x}", flush=True)

import bench  # noqa: E402
from distributed_gpu_test_amd.data import make_synthetic_data  # noqa: E402
from distributed_gpu_test_amd.models import SimpleNet  # noqa: E402
from distributed_gpu_test_amd.runtime.tiny_trainer import TinyMLPTrainer  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(42)
x, y = make_synthetic_data(2000, 20, 42)
tr = TinyMLPTrainer(SimpleNet(20, 64), x, y, 4, impl="fused", device=dev)
plan, counts = bench.build_plan(tr, 100000)
z = torch.zeros(16, device=dev)


def t(label, f, n=1000):
    for _ in range(50):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    dt = (time.perf_counter() - t0) / n * 1e6
    print(f"{mode:8s} {label:32s} {dt:7.2f} us", flush=True)


def trivial():
    z.add_(1)
    torch.cuda.synchronize()


t("trivial kernel + sync", trivial)
for k in (1, 10, 100):
    pk, ck = plan[:k].contiguous(), counts[:k].contiguous()

    def fused(pk=pk, ck=ck):
        tr.run_plan(pk, ck)
        torch.cuda.synchronize()
    t(f"fused K={k} + sync", fused, 500)
