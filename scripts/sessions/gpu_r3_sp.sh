#!/bin/bash
# 128x128 kernel: software-pipelined fragment reads (variant 5, five stages) vs front-loaded reads
# (variant 3, the default): numerics + bitwise tests, M = 1024 hot/cold, and the MLP step interleaved.
set -o pipefail
mkdir -p gpurun_out/sp
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_mlp_gemm.py > gpurun_out/sp/pytest.log 2>&1 || { tail -30 gpurun_out/sp/pytest.log; exit 1; }
tail -1 gpurun_out/sp/pytest.log
CHECK_VARIANT=5 VARIANTS=3,5 timeout -k 10 300 python scripts/bench_gemm_m1024.py > gpurun_out/sp/m1024.jsonl 2> gpurun_out/sp/m1024.err || { tail -20 gpurun_out/sp/m1024.err; exit 1; }
cat gpurun_out/sp/m1024.jsonl
for i in 1 2 3; do
  for v in 0 5; do
    DGT_GEMM_VARIANT=$v timeout -k 10 300 python bench.py --model mlp --steps 100 --warmup 10 --no-sweep > gpurun_out/sp/mlp_v${v}_$i.json 2> gpurun_out/sp/mlp_v${v}_$i.err || { tail -20 gpurun_out/sp/mlp_v${v}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/sp/mlp_v${v}_$i.json')); print('mlp variant $v run $i', d['value'], d['ms_per_step'])"
  done
done
