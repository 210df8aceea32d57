"""Fixed cost of one timed fused run (bias corrections in-kernel): host launch, device span, sync wake-up."""
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
plan, counts = bench.build_plan(tr, 100000)
pos = 0
for K in (1, 10, 100, 1000):
    rows = []
    for rep in range(6):
        p, c = plan[pos:pos + K], counts[pos:pos + K]
        pos += K
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        s.record()
        tr.run_plan(p, c)
        e.record()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rows.append((1e6 * (t1 - t0), 1e3 * s.elapsed_time(e), 1e6 * (t2 - t0)))
    r = rows[2:]
    avg = [sum(v[i] for v in r) / len(r) for i in range(3)]
    print(f"K={K:5d}: host launch {avg[0]:6.1f} us  device span {avg[1]:7.1f} us  total {avg[2]:7.1f} us  "
          f"(compute {K * 0.763:.1f} us)")
