#!/bin/bash
# fp32 64x64 tiles with two in-block k groups (8 waves) vs 4 waves, x split-K block target.
set -o pipefail
O=gpurun_out/r4f8
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_f32.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; exit $rc; }
run() {  # kg min_blocks
  DGT_F32_SMALL_KGROUPS=$1 DGT_F32_MIN_BLOCKS=$2 timeout -k 10 300 python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 50 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print('fp32 engine MLP kg $1 min_blocks $2', d['value'], d['ms_per_step'])" | tee -a $O/ab.txt
}
: > $O/ab.txt
for rep in 1 2; do
  run 2 256; run 2 512; run 2 1024; run 1 512
done
for kg in 2 1; do
  DGT_F32_SMALL_KGROUPS=$kg DGT_F32_MIN_BLOCKS=256 timeout -k 10 300 python scripts/bench_gemm_f32.py 1024x1024x1024 1000x1000x1000 256x4096x4096 > $O/gemm_kg$kg.jsonl 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
  echo "== kg $kg, min_blocks 256"; cat $O/gemm_kg$kg.jsonl
done
