#!/usr/bin/env python3
"""Where the driver-shape headline's fixed cost goes (1 GPU, fused kernel, K = 20).

For 300 repetitions each (medians, us): the bench's bracket (sync, launch, sync) through
``run_plan`` (the Python path: plan checks, stream lookup, ctypes call), the same launch with the
ctypes arguments prepared beforehand (``TinyMLPTrainer.bind_launch``: per-argument ctypes call + hipLaunchKernel, or the prepared
argument block + hipModuleLaunchKernel), a K = 1 launch, and the
platform floor (one tiny ``add_`` + sync).  The host part of each is reported separately."""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import build_plan  # noqa: E402
from distributed_gpu_test_amd.data import make_synthetic_data  # noqa: E402
from distributed_gpu_test_amd.models import SimpleNet  # noqa: E402
from distributed_gpu_test_amd.parallel import comm  # noqa: E402
from distributed_gpu_test_amd.runtime.tiny_trainer import TinyMLPTrainer  # noqa: E402

comm.init_distributed()
dev = torch.device("cuda", 0)
torch.manual_seed(42)
x, y = make_synthetic_data(2000, 20, 42)
tr = TinyMLPTrainer(SimpleNet(20, 64), x, y, 4, lr=1e-3, impl="fused", device=dev)
K, W, REPS = 20, 5, 300
plan, counts = build_plan(tr, W + K)
tr.reserve(K)
tp, tc = plan[W:], counts[W:]
for _ in range(20):
    tr.run_plan(tp, tc)
torch.cuda.synchronize()


def bracket(fn):
    host, total = [], []
    for _ in range(REPS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append(1e6 * (t1 - t0))
        total.append(1e6 * (t2 - t0))
    return {"host_us": round(statistics.median(host), 2), "total_us": round(statistics.median(total), 2),
            "p10_us": round(sorted(total)[REPS // 10], 2), "iters_per_s_at_median": round(K / statistics.median(total) * 1e6)}


one = torch.zeros(1, device=dev)
res = {"run_plan K=20": bracket(lambda: tr.run_plan(tp, tc))}
launch_args = tr.bind_launch(tp, tc, prepared=False)
res["bind_launch per-arg K=20"] = bracket(launch_args)
launch = tr.bind_launch(tp, tc)
res["bind_launch prepared K=20"] = bracket(launch)
# the bench's own sequence per repetition: a freshly bound launch, the held-back warmup step through
# its own bound launch, (optionally) the loss clone, sync, then the timed launch
def bench_like(clone: bool):
    host, total = [], []
    wp, wc = plan[W - 1:W], counts[W - 1:W]
    for _ in range(REPS // 3):
        launch_t = tr.bind_launch(tp, tc)
        tr.bind_launch(wp, wc)()
        if clone:
            tr.loss_acc.clone()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        launch_t()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append(1e6 * (t1 - t0))
        total.append(1e6 * (t2 - t0))
    return {"host_us": round(statistics.median(host), 2), "total_us": round(statistics.median(total), 2),
            "p10_us": round(sorted(total)[len(total) // 10], 2),
            "iters_per_s_at_median": round(K / statistics.median(total) * 1e6)}


res["bench sequence, loss clone"] = bench_like(True)
res["bench sequence, no clone"] = bench_like(False)
res["run_plan K=1"] = bracket(lambda: tr.run_plan(tp[:1], tc[:1]))
res["add_ floor"] = bracket(lambda: one.add_(1.0))
for k, v in res.items():
    print(json.dumps(dict(arm=k, **v)), flush=True)
tr.check()
