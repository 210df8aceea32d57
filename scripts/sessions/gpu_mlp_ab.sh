#!/bin/bash
# MLP trainer schedule A/B (flat / serial / overlap) + its GPU tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_mlp_gemm.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_mlp.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/mlp_ab.jsonl
for rep in 1 2; do
  for sch in flat serial overlap overlap-prio; do
    DGT_MLP_PRIO=$([ $sch = overlap-prio ] && echo 1 || echo 0) DGT_MLP_SCHEDULE=${sch%-prio} timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 > gpurun_out/ab_$sch.json 2> gpurun_out/ab_$sch.err || { tail -20 gpurun_out/ab_$sch.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_$sch.json')); print('$sch', d['value'], d['ms_per_step'])" | tee -a gpurun_out/mlp_ab.jsonl
  done
done
