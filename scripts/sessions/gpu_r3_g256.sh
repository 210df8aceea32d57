#!/bin/bash
# 256x256 GEMM: asm saddr DMAs (variant 7) and the Adam epilogue's state prefetch (variant 8) vs
# variant 2: tests, isolated timings, and the MLP step with the fused wgrad + Adam on each.
set -o pipefail
mkdir -p gpurun_out/g256
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_mlp_gemm.py -k "256 or adam or reference or identity or high_address" > gpurun_out/g256/pytest.log 2>&1 || { tail -30 gpurun_out/g256/pytest.log; exit 1; }
tail -1 gpurun_out/g256/pytest.log
VARIANTS=2,7,8 timeout -k 10 300 python scripts/bench_gemm256_ab.py > gpurun_out/g256/ab.jsonl 2> gpurun_out/g256/ab.err || { tail -20 gpurun_out/g256/ab.err; exit 1; }
cat gpurun_out/g256/ab.jsonl
for i in 1 2; do
  for v in 0 7 8; do
    DGT_MLP_WGA_VARIANT=$v timeout -k 10 300 python bench.py --model mlp --steps 50 --warmup 10 --no-sweep > gpurun_out/g256/mlp_v${v}_$i.json 2> gpurun_out/g256/mlp_v${v}_$i.err || { tail -20 gpurun_out/g256/mlp_v${v}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/g256/mlp_v${v}_$i.json')); print('mlp wga variant $v run $i', d['value'], d['ms_per_step'])"
  done
done
