#!/bin/bash
# fp32 64x64 GEMM with 1 K-tile in flight: gemm_f32 tests, fp32 engine MLP x3.

set -o pipefail
O=gpurun_out/r4p1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_f32.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for mb in 512; do
    DGT_F32_MIN_BLOCKS=$mb timeout -k 10 300 python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 50 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print('min_blocks $mb fp32 engine MLP', d['value'], d['ms_per_step'])" | tee -a $O/mlp.txt
  done
done
