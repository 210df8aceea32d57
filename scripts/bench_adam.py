#!/usr/bin/env python3
"""Fused-Adam bandwidth: the flat adam_flat kernel over the bench MLP's 67M parameters (fp32 master,
m, v, fp32 grads, bf16 param copy = 30 B/param), loop-shape variants interleaved in one process
(cdna_hip_programming.md §5.4 rule 24).  Prints one JSON line per variant."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_gpu_test_amd.ops.adam import adam_flat_  # noqa: E402

N = 4 * 4096 * 4096 + 4 * 4096 + 4096 + 1 + 3  # bench MLP, padded to a multiple of 4
VARIANTS = {0: "1 group, nontemporal, full grid (default)", 1: "2 groups, plain, grid<=4096",
            2: "2 groups, nontemporal, grid<=4096", 3: "1 group, plain, full grid",
            4: "8 elements per thread (16-byte 16-bit streams), nontemporal, full grid"}
GRAD_DTYPE = torch.bfloat16 if "bf16" in sys.argv[1:] else torch.float32  # the MLP trainer's grads are bf16
BYTES = 28 if GRAD_DTYPE == torch.bfloat16 else 30


def main():
    dev = torch.device("cuda")
    master = torch.randn(N, device=dev)
    grad = torch.randn(N, device=dev).to(GRAD_DTYPE)
    m = torch.zeros(N, device=dev)
    v = torch.zeros(N, device=dev)
    lp = torch.empty(N, device=dev, dtype=torch.bfloat16)
    times = {k: [] for k in VARIANTS}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    step = 0
    for rnd in range(5):
        for k in VARIANTS:
            torch.ops.dgt.adam_set_variant(k)
            for _ in range(3):
                step += 1
                adam_flat_(master, grad, m, v, step, 1e-4, param_lp=lp)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(10):
                step += 1
                adam_flat_(master, grad, m, v, step, 1e-4, param_lp=lp)
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 10 * 1e3)
    for k, name in VARIANTS.items():
        t = sorted(times[k])
        us = t[len(t) // 2]
        print(json.dumps({"variant": k, "desc": name, "grad": str(GRAD_DTYPE), "n_params": N, "us_median": round(us, 1), "us_min": round(t[0], 1),
                          "TBps": round(N * BYTES / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
