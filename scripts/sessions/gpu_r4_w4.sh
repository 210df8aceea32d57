#!/bin/bash
# 256x256 with 4 waves of 128x128 (variant 9) vs cross-phase prefetch (8): bitwise tests, hot timings.
set -o pipefail
O=gpurun_out/r4w4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mlp_gemm.py -x -q --timeout 120 --timeout-method thread -k "cross_phase or large_k_repeated" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; exit $rc; }
VARIANTS=8,9 REPS=2 timeout -k 10 300 python scripts/bench_gemm256_ab.py > $O/gemm256.jsonl 2> $O/gemm256.err || { tail -20 $O/gemm256.err; exit 1; }
cat $O/gemm256.jsonl
