#!/bin/bash
# MLP step: the shape rule (SP dgrad, FR forward) vs SP for the forward too (DGT_GEMM_VARIANT=5).
set -o pipefail
mkdir -p gpurun_out/spf
export TMPDIR=/tmp
for i in 1 2 3 4; do
  for v in 0 5; do
    DGT_GEMM_VARIANT=$v timeout -k 10 300 python bench.py --model mlp --steps 100 --warmup 10 --no-sweep > gpurun_out/spf/v${v}_$i.json 2> gpurun_out/spf/v${v}_$i.err || { tail -20 gpurun_out/spf/v${v}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/spf/v${v}_$i.json')); print('variant $v run $i', d['value'], d['ms_per_step'])"
  done
done
