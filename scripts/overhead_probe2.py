"""Fixed overhead of bench.timed_run's bracket at small K (1 GPU)."""
import time, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_gpu_test_amd.data import make_synthetic_data
from distributed_gpu_test_amd.models import SimpleNet
from distributed_gpu_test_amd.runtime.tiny_trainer import TinyMLPTrainer
dev = torch.device("cuda", 0)
torch.manual_seed(42)
x, y = make_synthetic_data(2000, 20, 42)
tr = TinyMLPTrainer(SimpleNet(20, 64), x, y, 4, impl="fused", device=dev)
plan, counts = tr.epoch_plan(1)
K, W = 10, 10
def bracket(zero_before_sync, check_status):
    tr.run_plan(plan[:W], counts[:W])
    torch.cuda.synchronize()
    if check_status:
        tr.check()
    if zero_before_sync:
        tr.loss_acc.zero_()
    torch.cuda.synchronize()
    if not zero_before_sync:
        tr.loss_acc.zero_()
    t0 = time.perf_counter()
    tr.run_plan(plan[W:W + K], counts[W:W + K])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6
for zb in (False, True):
    for cs in (True, False):
        ts = [bracket(zb, cs) for _ in range(8)]
        print(f"zero_before_sync={zb} check_status={cs}: " + " ".join(f"{t:.1f}" for t in ts))
