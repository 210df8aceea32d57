#!/usr/bin/env python3
"""Step time of the bf16 engine MLP (configs/ds_bench_mlp_bf16.json) with every bucket's collective
forced at world size 1 (DGT_FORCE_COLLECTIVES=1), for A/B of the reducer's launch paths:
DGT_REDUCER_NATIVE / DGT_REDUCER_THREAD, against the collective-free step
(``--no-force``).  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    force = "--no-force" not in sys.argv
    os.environ["DGT_FORCE_COLLECTIVES"] = "1" if force else "0"
    os.environ.setdefault("DGT_QUIET", "1")
    import torch
    from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
    from distributed_gpu_test_amd.parallel import comm
    from distributed_gpu_test_amd.runtime.engine_mlp import EngineMLPTrainer
    comm.init_distributed(backend="nccl")
    cfg = json.load(open(os.path.join(ROOT, "configs", "ds_bench_mlp_bf16.json")))
    torch.manual_seed(1234)
    tr = EngineMLPTrainer(SyntheticMLP(4096, 4), 1024, 8, cfg)
    plan, counts = tr.epoch_plan(1)
    for _ in range(20):
        tr.run_plan(plan[:1], counts[:1])
    torch.cuda.synchronize()
    n = 100
    t0 = time.perf_counter()
    for _ in range(n):
        tr.run_plan(plan[:1], counts[:1])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    r = tr.engine.reducer
    print(json.dumps({"force": force, "native": r.native is not None, "thread": r.launch_thread,
                      "side_concurrent": r.side_concurrent,
                      "ms_per_step": round(dt * 1e3, 4),
                      "iters_per_s": round(1 / dt, 1)}), flush=True)
    tr.close()
    comm.destroy()


if __name__ == "__main__":
    main()
