"""Where does the fixed per-run overhead of the fused bench go? (host timings, 1 GPU)"""
import time, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_gpu_test_amd.data import make_synthetic_data
from distributed_gpu_test_amd.models import SimpleNet
from distributed_gpu_test_amd.runtime.tiny_trainer import TinyMLPTrainer
from distributed_gpu_test_amd.ops import _ext
dev = torch.device("cuda", 0)
torch.manual_seed(42)
x, y = make_synthetic_data(2000, 20, 42)
tr = TinyMLPTrainer(SimpleNet(20, 64), x, y, 4, impl="fused", device=dev)
plan, counts = tr.epoch_plan(1)
tr.run_plan(plan, counts); torch.cuda.synchronize()
def timeit(name, fn, n=200):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n): fn()
    dt = (time.perf_counter() - t0) / n * 1e6
    print(f"{name:45s} {dt:8.1f} us")
timeit("torch.cuda.synchronize (idle)", torch.cuda.synchronize)
timeit("run_plan(1 step), no sync", lambda: tr.run_plan(plan[:1], counts[:1]))
timeit("run_plan(1 step) + sync", lambda: (tr.run_plan(plan[:1], counts[:1]), torch.cuda.synchronize()))
timeit("run_plan(10 steps) + sync", lambda: (tr.run_plan(plan[:10], counts[:10]), torch.cuda.synchronize()))
timeit("run_plan(100 steps) + sync", lambda: (tr.run_plan(plan[:100], counts[:100]), torch.cuda.synchronize()))
timeit("plan slicing", lambda: (plan[10:], counts[10:]))
e = torch.empty(1, device=dev)
timeit("tiny kernel launch (fill_) + sync", lambda: (e.fill_(1.0), torch.cuda.synchronize()))
ops = _ext.require()
timeit("op call only (1 step, no sync)", lambda: ops.tiny_mlp_train(tr.x, tr.y, plan[:1], counts[:1], tr.params, tr.exp_avg,
       tr.exp_avg_sq, tr.loss_acc, tr.status, 20, 64, 1e-3, 0.9, 0.999, 1e-8, 0.0, False, 1, [], 0, 1, 0, 0, 0))
# device-side duration of a 1-step and a 10-step launch
for n in (1, 10, 100):
    s, e2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record(); tr.run_plan(plan[:n], counts[:n]); e2.record(); torch.cuda.synchronize()
    print(f"device time run_plan({n})                       {s.elapsed_time(e2)*1e3:8.1f} us")
