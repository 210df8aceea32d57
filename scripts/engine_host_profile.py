"""Host-side profile of the generic engine's eager step on one GPU: cProfile over the DeepSpeed-API
loop (engine forward / backward / step on the reference SimpleNet, B = 4) after a warmup, top
functions by own time.  Where the eager engine's ~300 us/step of host work goes
(README: the eager engine is host-bound).

    python scripts/engine_host_profile.py [--steps 2000] [--config configs/ds_zero0.json]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DGT_QUIET", "1")

import torch  # noqa: E402

import bench  # noqa: E402
from distributed_gpu_test_amd.data import make_synthetic_data  # noqa: E402
from distributed_gpu_test_amd.models import SimpleNet  # noqa: E402
from distributed_gpu_test_amd.parallel import comm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--config", default=None)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--no-cprofile", action="store_true", help="only the unprofiled timings")
    a = ap.parse_args()
    comm.init_distributed()
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    torch.manual_seed(42)
    x, y = make_synthetic_data(2000, 20, 42)
    b = bench.DgtEngineBench(SimpleNet(20, 64), x, y, 4, dev, a.config)
    plan, counts = b.epoch_plan(0)
    reps = (a.steps + plan.shape[0] - 1) // plan.shape[0]
    plan, counts = plan.repeat(reps, 1)[:a.steps], counts.repeat(reps)[:a.steps]
    b.run_plan(plan[:200], counts[:200])
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    b.run_plan(plan, counts)
    t1 = time.perf_counter()  # the host has enqueued every step
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # enqueue ~= total: host-bound; total >> enqueue: the device (or its dispatch) is the limit
    print(f"[engine-host] impl={b.impl} {dt / a.steps * 1e6:.1f} us/step ({a.steps / dt:.0f} it/s) unprofiled, "
          f"host enqueue {(t1 - t0) / a.steps * 1e6:.1f} us/step")
    if a.no_cprofile:
        b.close()
        comm.destroy()
        return
    pr = cProfile.Profile()
    pr.enable()
    b.run_plan(plan, counts)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(a.top)
    b.close()
    comm.destroy()


if __name__ == "__main__":
    main()
