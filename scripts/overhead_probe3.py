"""bench.py's bracket after a long warmup: host time to launch, device time, first vs later runs."""
import time, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from distributed_gpu_test_amd.data import make_synthetic_data
from distributed_gpu_test_amd.models import SimpleNet
from distributed_gpu_test_amd.runtime.tiny_trainer import TinyMLPTrainer
dev = torch.device("cuda", 0)
torch.manual_seed(42)
x, y = make_synthetic_data(2000, 20, 42)
tr = TinyMLPTrainer(SimpleNet(20, 64), x, y, 4, impl="fused", device=dev)
W, K = int(sys.argv[1]), int(sys.argv[2])
plan, counts = bench.build_plan(tr, W + 5 * K)
tr.run_plan(plan[:W], counts[:W]); torch.cuda.synchronize(); tr.check()
for rep in range(5):
    p, c = plan[W + rep * K: W + (rep + 1) * K], counts[W + rep * K: W + (rep + 1) * K]
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s.record()
    tr.run_plan(p, c)
    e.record()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"W={W} K={K} rep {rep}: launch {1e6*(t1-t0):6.1f} us  total {1e6*(t2-t0):7.1f} us  device {1e3*s.elapsed_time(e):7.1f} us")
