#!/bin/bash
# 256x256 GEMM, cross-phase fragment prefetch (variant 8) vs the 8-phase kernel (2): bitwise tests,
# hot timings vs hipBLASLt, and the bf16 MLP step with the wgrad on 8 (interleaved).
set -o pipefail
O=gpurun_out/r4x
mkdir -p $O
echo "== pytest"
timeout -k 10 300 python -u -m pytest tests/test_mlp_gemm.py -x -q --timeout 120 --timeout-method thread -k "cross_phase or large_k_repeated or asm_staging" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; exit $rc; }
echo "== 256x256: 2 vs 8"
VARIANTS=2,8 REPS=2 timeout -k 10 300 python scripts/bench_gemm256_ab.py > $O/gemm256_xp.jsonl 2> $O/gemm256_xp.err || { tail -20 $O/gemm256_xp.err; exit 1; }
cat $O/gemm256_xp.jsonl
echo "== MLP step, wgrad variant 0 / 8"
: > $O/mlp_ab.txt
for rep in 1 2 3; do
for v in 0 8; do
  DGT_MLP_WGRAD_VARIANT=$v timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print('wgrad $v', d['value'], d['ms_per_step'], d['model_tflops'])" | tee -a $O/mlp_ab.txt
done
done
echo done
