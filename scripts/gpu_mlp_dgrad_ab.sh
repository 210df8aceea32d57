#!/bin/bash
# MLP: W^T refresh on the main stream vs a side stream (tests + interleaved bench).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_mlp_gemm.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_mlp.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for ts in nt kn; do
    DGT_MLP_DGRAD=$ts timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 > gpurun_out/ts.json 2> gpurun_out/ts.err || { tail -20 gpurun_out/ts.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ts.json')); print('dgrad=$ts', d['value'], d['ms_per_step'], d['model_tflops'])" | tee -a gpurun_out/mlp_tside.txt
  done
done
