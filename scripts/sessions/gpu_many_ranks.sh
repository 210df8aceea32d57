#!/bin/bash
# Multi-rank rehearsal on one GPU (gloo control plane): 4 and 8 ranks through the fused kernel's
# IPC exchange, and bench.py at 8 ranks.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_multiproc.py -x -v -m gpu -k "many_ranks or eight_ranks" -s --timeout 600 --timeout-method thread > gpurun_out/pytest_many.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|n_gpus" gpurun_out/pytest_many.log | tail -8; exit $rc
