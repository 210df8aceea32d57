#!/bin/bash
# MLP step A/B: per-layer bias row sums (DGT_MLP_BIAS_BATCH=0) vs one batched row sum over the
# layer-indexed g^T stack (default), interleaved, plus the MLP numerics tests and a kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mlp_gemm.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_mlp.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in 0 1; do
    DGT_MLP_BIAS_BATCH=$v timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 > gpurun_out/mlp_bb_$v.json 2> gpurun_out/mlp_bb_$v.err || { tail -20 gpurun_out/mlp_bb_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/mlp_bb_$v.json')); print('DGT_MLP_BIAS_BATCH=$v', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mlp_bb -o run -- python bench.py --model mlp --steps 20 --warmup 5 > gpurun_out/prof_mlp_bb.log 2>&1 || { tail -20 gpurun_out/prof_mlp_bb.log; exit 1; }
echo done
