"""Exact-fp32 GEMM small-grid split-K A/B (csrc/gemm_f32_kernel.h SPK): time gemm_f32 at the
engine MLP's batch-256 shapes under DGT_F32_SPLIT = 1 (off), 2, 4, 8 (caps; the shape rule picks
up to the cap), one subprocess per setting (the knob is read once per process).

  python scripts/bench_gemm_f32_split.py [--iters 200] > out.jsonl
"""
import argparse
import json
import os
import subprocess
import sys

SHAPES = [(256, 1024, 1024, 0, 0), (256, 1024, 1024, 0, 1), (128, 1024, 1024, 0, 0), (512, 1024, 1024, 0, 0),
          (256, 4096, 1024, 0, 0), (64, 1024, 4096, 0, 0)]


def child(iters: int) -> None:
    import torch
    from distributed_gpu_test_amd.ops import _ext
    ops = _ext.require()
    for M, N, K, la, lb in SHAPES:
        A = torch.randn(M, K, device="cuda")
        B = torch.randn(N, K, device="cuda") if lb == 0 else torch.randn(K, N, device="cuda")
        mask = torch.randn(M, K, device="cuda") if lb == 1 else None  # the dgrad form: masked A
        C = torch.empty(M, N, device="cuda")
        for _ in range(20):
            ops.gemm_f32(A, B, mask, None, C, la, lb, False, False)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            ops.gemm_f32(A, B, mask, None, C, la, lb, False, False)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        print(json.dumps({"split_cap": os.environ.get("DGT_F32_SPLIT"), "M": M, "N": N, "K": K, "la": la, "lb": lb,
                          "us": round(us, 2), "tflops": round(2.0 * M * N * K / us / 1e6, 1)}), flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        child(args.iters)
        return
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for cap in ("1", "2", "4", "8"):
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--iters", str(args.iters)],
                           env=dict(os.environ, DGT_F32_SPLIT=cap, PYTHONPATH=root), cwd=root, timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
