#!/bin/bash
# flat Adam loop shapes incl. the 8-element variant: numerics (bit-identical to the default), kernel
# bandwidth with fp32 and bf16 grads, and the bf16 MLP bench with the default vs variant 4 interleaved
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiny_mlp.py -x -q -m gpu -k "adam" --timeout 120 --timeout-method thread > gpurun_out/adam_v8_pytest.log 2>&1 || { tail -30 gpurun_out/adam_v8_pytest.log; exit 1; }
tail -1 gpurun_out/adam_v8_pytest.log
timeout -k 10 200 python scripts/bench_adam.py > gpurun_out/adam_v8_f32.jsonl 2>&1 && cat gpurun_out/adam_v8_f32.jsonl || exit 1
timeout -k 10 200 python scripts/bench_adam.py bf16 > gpurun_out/adam_v8_bf16.jsonl 2>&1 && cat gpurun_out/adam_v8_bf16.jsonl || exit 1
for r in 1 2 3; do
  for v in 0 4; do
    DGT_ADAM_VARIANT=$v timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 > gpurun_out/adam_v8_mlp_$v.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/adam_v8_mlp_$v.json')); print('variant $v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/adam_v8_mlp.txt
  done
done
