#!/usr/bin/env python3
"""Where does the whole-step graph's run-to-run spread come from?  

The DeepSpeed-API engine with ``configs/ds_graph_fused.json`` (the reference model, the whole step
as one captured graph launched as its kernels) measured 37.6k / 45.0k / 48.4k iters/s in three
processes of one session.  This probe times K steps of bench.py's DgtEngineBench loop and splits
each step into host time (the Python/C++ call that enqueues it: gather launch, copy, direct launch
or replay, engine bookkeeping) and device time (HIP events around the whole K-step region, plus the
device's busy time from a K-step region bracketed by events with the host far ahead), so one line
says whether a slow process waited on the device or on its own CPU.  ``--pin CPU`` pins the
process to one CPU first (``os.sched_setaffinity``: no exec, no launcher).

    python scripts/graph_variance_probe.py [--steps 4000] [--pin N]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4000)
    ap.add_argument("--config", default=os.path.join(ROOT, "configs", "ds_graph_fused.json"))
    ap.add_argument("--pin", type=int, default=None, help="pin the process to this CPU before anything else")
    ap.add_argument("--unpinned", action="store_true", help="the config's amd.pin_host_thread turned off")
    a = ap.parse_args()
    if a.pin is not None:
        os.sched_setaffinity(0, {a.pin})
    os.environ.setdefault("DGT_QUIET", "1")
    import torch
    import bench
    from distributed_gpu_test_amd.data import make_synthetic_data
    from distributed_gpu_test_amd.models import SimpleNet
    from distributed_gpu_test_amd.parallel import comm
    comm.init_distributed()
    torch.manual_seed(42)
    x, y = make_synthetic_data(2000, 20, 42)
    cfg = json.load(open(a.config))
    if a.unpinned:
        cfg.setdefault("amd", {})["pin_host_thread"] = False
    tr = bench.DgtEngineBench(SimpleNet(20, 64), x, y, 4, torch.device("cuda", 0), cfg)
    plan, counts = bench.build_plan(tr, a.steps + 200)
    tr.run_plan(plan[:200], counts[:200])
    torch.cuda.synchronize()
    plan_d = plan[200:].to(tr.device).long()
    batches = [plan_d[s, :c] for s, c in enumerate(counts[200:].tolist())]
    # (1) the host's enqueue time per step, and the end-to-end time
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    host = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    for rows in batches:
        h0 = time.perf_counter()
        tr.step(rows)
        host.append(time.perf_counter() - h0)
    e1.record()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    wall = t2 - t0
    dev = e0.elapsed_time(e1) / 1e3
    host.sort()
    n = len(host)
    # (2) device-only rate: a sleep kernel holds the stream while the host enqueues everything, then
    # the events bracket the device's own execution of the K steps (no host gaps inside)
    half = batches[: n // 2]
    torch.cuda.synchronize()
    torch.cuda._sleep(int(2e9 * 0.2))  # ~0.2 s of device spin at ~2 GHz: time to enqueue the steps
    f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f0.record()
    q0 = time.perf_counter()
    for rows in half:
        tr.step(rows)
    q1 = time.perf_counter()
    f1.record()
    torch.cuda.synchronize()
    dev_only = f0.elapsed_time(f1) / 1e3
    out = {"config": os.path.basename(a.config), "impl": tr.impl, "pin": a.pin, "engine_pin": tr.engine.host_cpu,
           "steps": n,
           "iters_per_s": round(n / wall, 1), "us_per_step": round(1e6 * wall / n, 2),
           "host_enqueue_us_mean": round(1e6 * sum(host) / n, 2),
           "host_enqueue_us_p50": round(1e6 * host[n // 2], 2), "host_enqueue_us_p90": round(1e6 * host[int(n * 0.9)], 2),
           "host_loop_us_per_step": round(1e6 * (t1 - t0) / n, 2),
           "device_span_us_per_step": round(1e6 * dev / n, 2),
           "device_only_us_per_step": round(1e6 * dev_only / len(half), 2),
           "enqueue_ahead_us_per_step": round(1e6 * (q1 - q0) / len(half), 2),
           "cpus_allowed": len(os.sched_getaffinity(0))}
    print(json.dumps(out), flush=True)
    tr.close()
    comm.destroy()


if __name__ == "__main__":
    main()
