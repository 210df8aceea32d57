#!/bin/bash
# Fused wgrad+Adam epilogue batching A/B: numerics tests, isolated layer timing, MLP step vs _ab/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mlp_gemm.py -x -q -m gpu --timeout 120 --timeout-method thread -k "adam or fused" > gpurun_out/pytest_adam_epi.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_adam_epi.log; [ $rc -eq 0 ] || exit $rc
for t in _ab .; do
  (cd $t && timeout -k 10 200 python scripts/bench_wgrad_adam.py > /tmp/wa.txt 2>&1) || { tail -5 /tmp/wa.txt; exit 1; }
  echo "== $t"; grep -i "fused variant 0\|flat Adam\|wgrad GEMM" /tmp/wa.txt
done
bash scripts/gpu_ab_mlp_tree.sh
