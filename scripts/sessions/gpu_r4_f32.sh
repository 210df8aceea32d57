#!/bin/bash
# fp32 MFMA GEMM: numerics tests, hot timings vs hipBLASLt, and a rocprofv3 kernel trace of the
# DeepSpeed-API engine on a fp32 SyntheticMLP(1024, 4) at batch 1024 (no Cijk_* kernels expected).
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp
echo "== pytest test_gemm_f32"
timeout -k 10 400 python -u -m pytest tests/test_gemm_f32.py -x -q --timeout 120 --timeout-method thread > $O/pytest_f32.log 2>&1; rc=$?
tail -3 $O/pytest_f32.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest_f32.log | head -20; exit $rc; }
echo "== gemm_f32 vs hipBLASLt"
timeout -k 10 300 python scripts/bench_gemm_f32.py > $O/gemm_f32.jsonl 2> $O/gemm_f32.err || { tail -20 $O/gemm_f32.err; exit 1; }
cat $O/gemm_f32.jsonl
echo "== engine fp32 MLP bench"
timeout -k 10 300 python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 50 --warmup 10 > $O/bench_mlp_fp32.json 2> $O/bench_mlp_fp32.err || { tail -20 $O/bench_mlp_fp32.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_mlp_fp32.json')); print(d['value'], d['ms_per_step'], d['model_tflops'], d['dtype'], d['config']['impl'])"
echo "== rocprof engine fp32 MLP"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp_fp32 -o run -- python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 20 --warmup 5 --no-sweep > $O/prof_mlp_fp32.log 2>&1 || { tail -20 $O/prof_mlp_fp32.log; exit 1; }
find $O/prof_mlp_fp32 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/mlp_fp32_kernel_stats.csv
cut -d, -f1-4 $O/mlp_fp32_kernel_stats.csv | head -20
echo done
