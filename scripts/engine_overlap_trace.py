#!/usr/bin/env python3
"""Does the engine's gradient collective overlap backward?  

``run``: the bf16 engine MLP (``configs/ds_bench_mlp_bf16.json``: SyntheticMLP(4096, 4), batch 1024,
fp32 wire, per-layer buckets) through the DeepSpeed-style API at world size 1 with
``DGT_FORCE_COLLECTIVES=1``: ProcessGroupNCCL (RCCL) runs every bucket's all-reduce on its own
stream exactly as at N > 1 (a 1-rank sum: RCCL's copy kernels), and the fused MFMA chain reports
each layer complete from inside its backward (``ops.linear.grad_ready``).  Run it under
``rocprofv3 --kernel-trace`` and then

``analyze CSV``: for the last steady-state step, the compute stream's backward kernels in order and,
for every kernel of another stream (the wire cast, RCCL's kernels), the compute kernel that was
running when it started -- the first collective kernel must start before the last dgrad GEMM ends.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 scripts/engine_overlap_trace.py run
    python3 scripts/engine_overlap_trace.py analyze OUT/run_kernel_trace.csv
"""
from __future__ import annotations

import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(steps: int = 12) -> None:
    os.environ["DGT_FORCE_COLLECTIVES"] = "1"
    os.environ.setdefault("DGT_QUIET", "1")
    import torch
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.parallel import comm
    from distributed_gpu_test_amd.runtime.engine_mlp import EngineMLPTrainer
    comm.init_distributed(backend="nccl")
    cfg = json.load(open(os.path.join(ROOT, "configs", "ds_bench_mlp_bf16.json")))
    cfg.pop("train_batch_size", None)
    torch.manual_seed(1234)
    tr = EngineMLPTrainer(SyntheticMLP(4096, 4), 1024, 8, cfg)
    plan, counts = tr.epoch_plan(1)
    for _ in range(steps):
        tr.run_plan(plan[:1], counts[:1])
    torch.cuda.synchronize()
    e = tr.engine
    print(json.dumps({"steps": steps, "buckets": [[b.start, b.numel, b.params] for b in e.layout.buckets],
                      "layer_notifications": e.layer_notifications, "fused_layers": e.fused_linear_layers,
                      "thread_launches": e.reducer.thread_launches, "native_launches": e.reducer.native_launches,
                      "reducer_thread": e.reducer.launch_thread, "native": e.reducer.native is not None,
                      "side_concurrent": e.reducer.side_concurrent,
                      "bytes_reduced": e.reducer.bytes_reduced}), flush=True)
    tr.close()
    comm.destroy()


def analyze(path: str) -> None:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    for r in rows:
        r["t0"], r["t1"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    adam = [r for r in rows if "adam_flat_kernel" in r["Kernel_Name"]]
    if len(adam) < 3:
        sys.exit("fewer than 3 Adam launches in the trace")
    compute = adam[-1]["Stream_Id"]
    # the last full step: after the second-to-last Adam, up to and including the last one
    lo, hi = adam[-2]["t1"], adam[-1]["t1"]
    step = [r for r in rows if lo < r["t0"] <= hi]
    comp = [r for r in step if r["Stream_Id"] == compute]
    other = [r for r in step if r["Stream_Id"] != compute]
    gemms = [r for r in comp if "gemm" in r["Kernel_Name"]]
    # the backward's GEMMs follow the forward's (4 MFMA layers): fwd = first 4, then wgrad/dgrad pairs
    bwd = gemms[4:]
    t_base = comp[0]["t0"]
    print(f"compute stream {compute}: {len(comp)} kernels in the last step; other streams: {len(other)} kernels")
    print("compute stream, in order (us from step start):")
    for r in comp:
        print(f"  {(r['t0'] - t_base) / 1e3:8.1f} .. {(r['t1'] - t_base) / 1e3:8.1f}  {r['Kernel_Name'][:90]}")
    print("other streams (start, the compute kernel running then):")
    for r in other:
        run_ = [c for c in comp if c["t0"] <= r["t0"] < c["t1"]]
        where = run_[0]["Kernel_Name"][:60] if run_ else "(compute idle)"
        print(f"  stream {r['Stream_Id']:>3} {(r['t0'] - t_base) / 1e3:8.1f} .. {(r['t1'] - t_base) / 1e3:8.1f}  "
              f"{r['Kernel_Name'][:45]:45s}  during {where}")
    last_bwd_gemm_end = max(r["t1"] for r in bwd) if bwd else None
    # RCCL's kernels (a 1-rank in-place all-reduce launches none) and the wire casts the reducer issues
    # on the side stream immediately before each bucket's collective (the collective's launch point)
    coll = [r for r in other if "rocclr" in r["Kernel_Name"] or "nccl" in r["Kernel_Name"].lower()
            or "elementwise" in r["Kernel_Name"]]
    if coll and last_bwd_gemm_end is not None:
        first = min(r["t0"] for r in coll)
        before = sum(1 for r in coll if r["t0"] < last_bwd_gemm_end)
        print(f"first collective-stream kernel at {(first - t_base) / 1e3:.1f} us; last backward GEMM ends at "
              f"{(last_bwd_gemm_end - t_base) / 1e3:.1f} us; {before} of {len(coll)} collective kernels start before "
              f"it -> overlap {'YES' if first < last_bwd_gemm_end else 'NO'}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "analyze":
        analyze(sys.argv[2])
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 12)
