#!/bin/bash
# fp32 64x64 GEMM compiled for 2 blocks per CU with 2 K-tiles in flight (isolates the launch bound): fp32 engine MLP x3.

set -o pipefail
O=gpurun_out/r4lb2
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for mb in 512; do
    DGT_F32_MIN_BLOCKS=$mb timeout -k 10 300 python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 50 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print('min_blocks $mb fp32 engine MLP', d['value'], d['ms_per_step'])" | tee -a $O/mlp.txt
  done
done
