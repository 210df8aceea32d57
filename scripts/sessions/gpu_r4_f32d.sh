#!/bin/bash
# fp32 GEMM 128x128 blocks: 8 waves (default now) vs 4 (DGT_F32_BIG_THREADS=256): numerics tests,
# microbench vs hipBLASLt on the big shapes, fp32 engine MLP.
set -o pipefail
O=gpurun_out/r4f4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_f32.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; exit $rc; }
for t in 512 256; do
  echo "== threads $t"
  DGT_F32_BIG_THREADS=$t timeout -k 10 300 python scripts/bench_gemm_f32.py 4096x4096x4096 8192x8192x8192 2048x2048x2048 1024x4096x4096 > $O/gemm_t$t.jsonl 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
  cat $O/gemm_t$t.jsonl
done
timeout -k 10 300 python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 50 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print('fp32 engine MLP', d['value'], d['ms_per_step'])"
