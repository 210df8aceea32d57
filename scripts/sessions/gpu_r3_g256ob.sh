#!/bin/bash
# 256x256 kernel: one barrier per phase (variant 5) vs two (variant 2): bitwise tests, isolated A/B.
set -o pipefail
mkdir -p gpurun_out/pb
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_mlp_gemm.py -k "256 or variant5 or identity" > gpurun_out/pb/pytest.log 2>&1 || { tail -30 gpurun_out/pb/pytest.log; exit 1; }
tail -1 gpurun_out/pb/pytest.log
REPS=3 VARIANTS=2,5 timeout -k 10 300 python scripts/bench_gemm256_ab.py > gpurun_out/pb/ab.jsonl 2> gpurun_out/pb/ab.err || { tail -20 gpurun_out/pb/ab.err; exit 1; }
cat gpurun_out/pb/ab.jsonl
