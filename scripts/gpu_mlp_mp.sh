#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_mlp_gemm.py tests/test_gpu_multiproc.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_mlp_mp.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_mlp_mp.log; exit $rc
