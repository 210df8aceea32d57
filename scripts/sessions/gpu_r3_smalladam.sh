#!/bin/bash
# Small-region reduction + Adam in one launch: MLP/GEMM tests, MLP step interleaved vs _ab/.
set -o pipefail
mkdir -p gpurun_out/sa
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_mlp_gemm.py > gpurun_out/sa/pytest.log 2>&1 || { tail -30 gpurun_out/sa/pytest.log; exit 1; }
tail -1 gpurun_out/sa/pytest.log
rm -f gpurun_out/ab_mlp_tree.txt
bash scripts/gpu_ab_mlp_tree.sh && cp gpurun_out/ab_mlp_tree.txt gpurun_out/sa/
