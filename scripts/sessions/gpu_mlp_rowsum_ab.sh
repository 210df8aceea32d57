#!/bin/bash
# bf16 MLP step: bias-gradient row sums on a side stream beside the dgrad (DGT_MLP_ROWSUM_SIDE=1,
# default) vs in line (0); interleaved fresh-process runs, REPS each; plus the fused-path tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mlp_gemm.py -k "fused_adam or trainer" > gpurun_out/rs_tests.log 2>&1; rc=$?; tail -1 gpurun_out/rs_tests.log; [ $rc -eq 0 ] || exit $rc
for r in $(seq ${REPS:-3}); do
  for v in 0 1; do
    DGT_MLP_ROWSUM_SIDE=$v timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 > gpurun_out/rs.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/rs.json').read().splitlines()[-1]); print('rowsum_side=$v', d['value'], round(d['ms_per_step'], 4))"
  done
done
