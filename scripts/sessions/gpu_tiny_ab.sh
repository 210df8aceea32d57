#!/bin/bash
# Fused tiny-MLP kernel: step-ordered (DGT_TINY_PIPE=0) vs software-pipelined loop, tests + A/B bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny_mlp.py tests/test_gpu_multiproc.py -x -q -m gpu -k "not eight_ranks" --timeout 300 --timeout-method thread > gpurun_out/pytest_tiny.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_tiny.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/tiny_ab.txt
for rep in 1 2 3; do
  for p in 0 1; do
    DGT_TINY_PIPE=$p timeout -k 10 120 python bench.py --steps 200000 --warmup 5000 > gpurun_out/tab.json 2> gpurun_out/tab.err || { tail -20 gpurun_out/tab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/tab.json')); print('pipe=$p', d['value'], round(d['ms_per_step']*1e3,4), 'us/step', d['mean_loss'])" | tee -a gpurun_out/tiny_ab.txt
  done
done
