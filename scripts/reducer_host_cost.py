#!/usr/bin/env python3
"""Host cost of one gradient-bucket launch of the engine's reducer (ProcessGroupNCCL = RCCL).

The engine MLP's overlap trace (profiles/r6_engine_overlap_trace.txt) showed the compute stream idle
between layers while the host issued each layer's bucket: the per-layer launch is on the same host
thread that enqueues the next layer's GEMMs.  This times, per call on the host (mean / p50 / p90 us):

* ``event``: record a HIP event on the compute stream (what a hand-off to another thread costs);
* ``cast``: side.wait_stream + the bf16 -> fp32 wire cast launched on the side stream;
* ``allreduce``: ``dist.all_reduce(async_op=True)`` of a 16.8M-element fp32 bucket;
* ``launch``: GradReducer._launch of such a bucket (cast + all-reduce + bookkeeping);
* ``native_submit``: the same bucket handed to the native C++ launcher (csrc/bucket_launcher.cpp).

World size 1 with DGT_FORCE_COLLECTIVES=1 (a 1-rank RCCL communicator), as the trace ran.
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def stats(xs):
    xs = sorted(xs)
    n = len(xs)
    return {"mean": round(1e6 * sum(xs) / n, 2), "p50": round(1e6 * xs[n // 2], 2), "p90": round(1e6 * xs[int(0.9 * n)], 2)}


def main():
    os.environ["DGT_FORCE_COLLECTIVES"] = "1"
    import torch
    import torch.distributed as dist
    from distributed_gpu_test_amd.parallel import comm
    from distributed_gpu_test_amd.parallel.reducer import GradReducer
    from distributed_gpu_test_amd.runtime.flat import FlatLayout
    comm.init_distributed(backend="nccl")
    dev = torch.device("cuda", 0)
    n = 16781312
    out = {}
    cur = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    src = torch.randn(n, device=dev).to(torch.bfloat16)
    dst = torch.empty(n, device=dev)
    for _ in range(5):
        dist.all_reduce(dst)
    torch.cuda.synchronize()
    t = []
    for _ in range(200):
        t0 = time.perf_counter()
        ev = torch.cuda.Event()
        ev.record(cur)
        t.append(time.perf_counter() - t0)
    out["event"] = stats(t)
    t = []
    for _ in range(100):
        t0 = time.perf_counter()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            dst.copy_(src)
        t.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    out["cast"] = stats(t)
    t, works = [], []
    for _ in range(100):
        t0 = time.perf_counter()
        works.append(dist.all_reduce(dst, async_op=True))
        t.append(time.perf_counter() - t0)
    for w in works:
        w.wait()
    torch.cuda.synchronize()
    out["allreduce"] = stats(t)
    layout = FlatLayout([(4096, 4096), (4096,)] * 4, 8 << 20, 1, units=[[0, 1], [2, 3], [4, 5], [6, 7]])
    grad = torch.zeros(layout.total, dtype=torch.bfloat16, device=dev)
    red = GradReducer(grad, layout, 0, 1, 0, comm_dtype=torch.float32)
    t = []
    for _ in range(25):
        red.arm(True)
        for bi in range(len(layout.buckets)):
            t0 = time.perf_counter()
            red._launch(bi)
            t.append(time.perf_counter() - t0)
        red.finish()
    torch.cuda.synchronize()
    out["launch"] = stats(t)
    red.close()
    # the native launcher: the backward thread's cost is the submit (event record + queue push)
    from distributed_gpu_test_amd.parallel.rccl import RcclComm
    red = GradReducer(grad, layout, 0, 1, 0, comm_dtype=torch.float32, native_comm=RcclComm(dev))
    assert red.native is not None
    t = []
    for _ in range(25):
        red.arm(True)
        for bi in range(len(layout.buckets)):
            t0 = time.perf_counter()
            red._launch(bi)
            t.append(time.perf_counter() - t0)
        red.finish()
    torch.cuda.synchronize()
    out["native_submit"] = stats(t)
    out["native_launches"] = red.native_launches
    red.close()
    print(json.dumps(out), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
