"""Where the time of bench.py's short timed region goes (driver shape: --steps 20 --warmup 5).

Replays bench.timed_run's bracket R times in ONE process and splits each run into: host launch
(run_plan returns), device wait (synchronize returns), closing barrier + sync.  Variants:
  one  : warmup as ONE launch of W steps (bench.py today)
  split: warmup as W launches of 1 step (the launch path is hot W times before the bracket)
Usage: python scripts/bench_bracket_probe.py [K] [W] [R]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from distributed_gpu_test_amd.data import make_synthetic_data  # noqa: E402
from distributed_gpu_test_amd.models import SimpleNet  # noqa: E402
from distributed_gpu_test_amd.parallel import comm  # noqa: E402
from distributed_gpu_test_amd.runtime.tiny_trainer import TinyMLPTrainer  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
W = int(sys.argv[2]) if len(sys.argv) > 2 else 5
R = int(sys.argv[3]) if len(sys.argv) > 3 else 8
comm.init_distributed()
dev = torch.device("cuda", 0)


def one_run(split: bool):
    torch.manual_seed(42)
    x, y = make_synthetic_data(2000, 20, 42)
    tr = TinyMLPTrainer(SimpleNet(20, 64), x, y, 4, impl="fused", device=dev)
    plan, counts = bench.build_plan(tr, W + K)
    if split:
        for s in range(W):
            tr.run_plan(plan[s:s + 1], counts[s:s + 1])
    else:
        tr.run_plan(plan[:W], counts[:W])
    torch.cuda.synchronize()
    tr.check()
    tp, tc = plan[W:], counts[W:]
    tr.loss_acc.zero_()
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.run_plan(tp, tc)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    comm.barrier()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    tr.close()
    return 1e6 * (t1 - t0), 1e6 * (t2 - t1), 1e6 * (t3 - t2), 1e6 * (t3 - t0)


for variant in ("one", "split", "one", "split"):
    rows = [one_run(variant == "split") for _ in range(R)]
    tot = sorted(r[3] for r in rows)
    print(f"{variant:5s} K={K} W={W}: first {rows[0][3]:6.1f} us  median {tot[len(tot) // 2]:6.1f}  min {tot[0]:6.1f}"
          f"  | median launch {sorted(r[0] for r in rows)[R // 2]:5.1f}  wait {sorted(r[1] for r in rows)[R // 2]:5.1f}"
          f"  close {sorted(r[2] for r in rows)[R // 2]:4.1f}  -> {K / (tot[len(tot) // 2] * 1e-6):,.0f} it/s",
          flush=True)
