"""First-launch host latency after a synchronize: blocking sync vs spin-query before the bracket."""
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
W, K = 20000, 100
plan, counts = bench.build_plan(tr, W + 40 * K)
tr.reserve(W)
def spin():
    st = torch.cuda.current_stream()
    while not st.query():
        pass
for mode in ("sync", "spin", "sync", "spin"):
    tr.run_plan(plan[:W], counts[:W])
    if mode == "spin":
        spin()
    torch.cuda.synchronize()
    tr.check()
    if mode == "spin":
        # keep the host path hot: a few no-op launches, spin, then the contract's synchronize
        for _ in range(3):
            tr.loss_acc.add_(0.0)
        spin()
    torch.cuda.synchronize()
    p, c = plan[W:W + K], counts[W:W + K]
    t0 = time.perf_counter()
    tr.run_plan(p, c)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{mode}: launch {1e6*(t1-t0):6.1f} us  total {1e6*(t2-t0):7.1f} us")
