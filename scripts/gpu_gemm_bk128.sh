#!/bin/bash
# BK = 128 gemm (variant 7): numerics tests, the M = 1024 products per kernel (hot / cold), and the
# bf16 MLP step with the forward + dgrad on variant 7 vs the shape-picked default, interleaved
# fresh-process runs, REPS each.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mlp_gemm.py -k "gemm" > gpurun_out/bk_tests.log 2>&1; rc=$?; tail -1 gpurun_out/bk_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_gemm_m1024.py > gpurun_out/bk_m1024.jsonl 2>&1 || exit 1
cat gpurun_out/bk_m1024.jsonl
for r in $(seq ${REPS:-3}); do
  for v in 0 7 8; do
    DGT_MLP_GEMM_VARIANT=$v timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 > gpurun_out/bk.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/bk.json').read().splitlines()[-1]); print('gemm_variant=$v', d['value'], round(d['ms_per_step'], 4))"
  done
done
