"""Host-side costs of one timed run of the fused kernel (lean launcher vs torch op dispatch, stream lookup,
synchronize).  NOTE: the raw launches below keep re-running step 0 on the trainer's state."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from distributed_gpu_test_amd.data import make_synthetic_data
from distributed_gpu_test_amd.models import SimpleNet
from distributed_gpu_test_amd.runtime.tiny_trainer import TinyMLPTrainer
from distributed_gpu_test_amd.ops import _ext
dev = torch.device("cuda", 0)
torch.manual_seed(42)
x, y = make_synthetic_data(2000, 20, 42)
tr = TinyMLPTrainer(SimpleNet(20, 64), x, y, 4, impl="fused", device=dev)
plan, counts = bench.build_plan(tr, 100000)
def t(label, f, n=2000):
    for _ in range(50): f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n): f()
    dt = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    print(f"{label:40s} {dt:7.2f} us", flush=True)
p1, c1 = plan[:1].contiguous(), counts[:1].contiguous()
t("current_stream().cuda_stream", lambda: torch.cuda.current_stream(dev).cuda_stream)
t("slice plan[1:]", lambda: plan[1:])
s = torch.cuda.current_stream(dev).cuda_stream
t("run_plan K=1 (lean ctypes launcher)", lambda: tr.run_plan(p1, c1), 500)
from distributed_gpu_test_amd.runtime.tiny_trainer import _raw_stream
t("_raw_stream", lambda: _raw_stream(0))
t("_lean_ok checks", lambda: tr._lean_ok(p1, c1, 1))
lib, lh = _ext.c_lib(), tr._lh
pp, cp = p1.data_ptr(), c1.data_ptr()
tr.reserve(1)
wp = tr._ws_ptr
t("dgt_tiny_launch (raw ctypes call)", lambda: lib.dgt_tiny_launch(lh, pp, cp, 1, 4, 0, 0, wp), 500)
ops = _ext.require()
def old():
    ops.tiny_mlp_train(tr.x, tr.y, p1, c1, tr.params, tr.exp_avg, tr.exp_avg_sq, tr.loss_acc, tr.status, 20, 64,
                       1e-3, 0.9, 0.999, 1e-8, 0.0, False, 0, [], 0, 1, 0, 0, 0, -1, tr._ws)
t("torch op tiny_mlp_train K=1", old, 500)
t("synchronize (idle)", lambda: torch.cuda.synchronize())
e = torch.cuda.Event(enable_timing=True)
t("event.record", lambda: e.record())
def launch_sync():
    old()
    torch.cuda.synchronize()
t("fused launch + synchronize K=1", launch_sync, 500)
z = torch.zeros(1, device=dev)
def tiny_kernel_sync():
    z.add_(1)
    torch.cuda.synchronize()
t("torch add_ + synchronize", tiny_kernel_sync, 500)
