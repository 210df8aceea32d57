#!/bin/bash
# 256 x 256 single-barrier gemm (variant 9): numerics, the K = 1024 weight gradient per kernel, and the
# bf16 MLP step with its fused wgrad + Adam on variant 9 vs the shape-picked default.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mlp_gemm.py -k "gemm" > gpurun_out/g9_tests.log 2>&1; rc=$?; tail -1 gpurun_out/g9_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_gemm_wgrad.py 2>&1 | grep -v amdgpu.ids || exit 1
for r in $(seq ${REPS:-3}); do
  for v in 0 9; do
    DGT_MLP_FUSED_VARIANT=$v timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 > gpurun_out/g9.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/g9.json').read().splitlines()[-1]); print('fused_variant=$v', d['value'], round(d['ms_per_step'], 4))"
  done
done
