"""Per-call host time of the DeepSpeed-API loop on the reference SimpleNet (B = 4, fp32): the batch
gather (data.gather_batch), ``engine(x)``, the loss, ``engine.backward`` and ``engine.step``, each bracketed by
perf_counter (no profiler), plus the HIP graph replays inside them.  Shows which call's host cost
moves when the graph_module path runs slower in one process than in another.

    python scripts/engine_step_breakdown.py [--steps 3000] [--config configs/ds_graph_module.json]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DGT_QUIET", "1")

import torch  # noqa: E402

import bench  # noqa: E402
from distributed_gpu_test_amd.data import gather_batch, make_synthetic_data  # noqa: E402
from distributed_gpu_test_amd.models import SimpleNet  # noqa: E402
from distributed_gpu_test_amd.ops import BCEWithLogitsLoss  # noqa: E402
from distributed_gpu_test_amd.parallel import comm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--config", default="configs/ds_graph_module.json")
    ap.add_argument("--side-stream", action="store_true", help="run the loop on a created stream")
    ap.add_argument("--torch-loss", action="store_true",
                    help="torch.nn.BCEWithLogitsLoss (the reference's criterion: autograd backward, no graphed tail)")
    a = ap.parse_args()
    comm.init_distributed()
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    x, y = make_synthetic_data(2000, 20, 42)
    b = bench.DgtEngineBench(SimpleNet(20, 64), x, y, 4, dev, a.config or None)
    eng = b.engine
    crit = torch.nn.BCEWithLogitsLoss() if a.torch_loss else BCEWithLogitsLoss(sum_into=b.loss_acc)
    plan, counts = b.epoch_plan(0)
    reps = (a.steps + plan.shape[0] - 1) // plan.shape[0]
    plan = plan.repeat(reps, 1)[:a.steps].to(dev).long()
    rows_l = [plan[s, :4] for s in range(a.steps)]
    replay_t = [0.0, 0]
    orig = torch.cuda.CUDAGraph.replay

    def timed_replay(self):
        t = time.perf_counter()
        orig(self)
        replay_t[0] += time.perf_counter() - t
        replay_t[1] += 1

    names = ("gather", "forward", "loss", "backward", "step")
    if a.side_stream:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        torch.cuda.set_stream(side)
    for phase in ("warm", "timed"):
        acc = [0.0] * 5
        replay_t[0], replay_t[1] = 0.0, 0
        torch.cuda.CUDAGraph.replay = timed_replay if phase == "timed" else orig
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        ptrs = []
        for rows in (rows_l[:300] if phase == "warm" else rows_l):
            t0 = time.perf_counter()
            xb, yb = gather_batch(rows, b.x, b.y)
            if len(ptrs) < 16:
                ptrs.append(xb.data_ptr())
            t1 = time.perf_counter()
            z = eng(xb)
            t2 = time.perf_counter()
            loss = crit(z.float(), yb)
            t3 = time.perf_counter()
            eng.backward(loss)
            t4 = time.perf_counter()
            eng.step()
            t5 = time.perf_counter()
            acc[0] += t1 - t0
            acc[1] += t2 - t1
            acc[2] += t3 - t2
            acc[3] += t4 - t3
            acc[4] += t5 - t4
        t_enq = time.perf_counter()
        torch.cuda.synchronize()
        t_end = time.perf_counter()
    torch.cuda.CUDAGraph.replay = orig
    n = a.steps
    us = lambda v: f"{v / n * 1e6:.1f}"  # noqa: E731
    print(f"[breakdown] {'side stream ' if a.side_stream else ''}{'torch loss ' if a.torch_loss else ''}impl={b.impl} total {us(t_end - t_start)} us/step, enqueue {us(t_enq - t_start)}; "
          + ", ".join(f"{k} {us(v)}" for k, v in zip(names, acc))
          + f"; graph replays {replay_t[1] / n:.1f}/step {us(replay_t[0])} us/step", flush=True)
    base = min(ptrs)
    print(f"[breakdown] batch addresses (offsets): {[p - base for p in ptrs]}")
    for fn in eng._graphed_fwd.values():
        print(f"[breakdown] copying-graph replays {fn.replays}, bound {[r.replays for r in fn.bound.values()]}, "
              f"evictions {fn.evictions}"
              f"{' bind failed: ' + fn.bind_failed if fn.bind_failed else ''}", flush=True)
    b.close()
    comm.destroy()


if __name__ == "__main__":
    main()
