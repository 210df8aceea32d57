#!/bin/bash
# fp32: vectorized split-K reduce + unrolled bias-gradient column sums: tests, engine MLP x3, stats.
set -o pipefail
O=gpurun_out/r4f7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_f32.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 50 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print('fp32 engine MLP', d['value'], d['ms_per_step'])"
done
for mb in 256 512; do
  DGT_F32_MIN_BLOCKS=$mb timeout -k 10 300 python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 50 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print('fp32 engine MLP min_blocks $mb', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 20 --warmup 5 --no-sweep > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
cut -d, -f1-4 $O/kernel_stats.csv | head -12
