#!/bin/bash
# Kernel stats of the final tree's engine MLPs (fp32 and bf16 through the DeepSpeed-API engine).
set -o pipefail
O=gpurun_out/r4fp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p32 -o run -- python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 20 --warmup 5 --no-sweep > $O/p32.log 2>&1 || { tail -20 $O/p32.log; exit 1; }
find $O/p32 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/fp32_engine_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p16 -o run -- python bench.py --model mlp --impl dgt-engine --steps 20 --warmup 5 --no-sweep > $O/p16.log 2>&1 || { tail -20 $O/p16.log; exit 1; }
find $O/p16 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/bf16_engine_kernel_stats.csv
cut -d, -f1-3 $O/fp32_engine_kernel_stats.csv | head -14
cut -d, -f1-3 $O/bf16_engine_kernel_stats.csv | head -14
