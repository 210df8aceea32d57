#!/bin/bash
# fp32 with the dgrad output mask: diag + engine MLP x3 + kernel stats (tests ran in the gate).
set -o pipefail
O=gpurun_out/r4f10
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python scripts/diag_f32_engine.py > $O/diag.txt 2>&1 || { tail -20 $O/diag.txt; exit 1; }
grep -v "amdgpu.ids\|destroy_process" $O/diag.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 50 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print('fp32 engine MLP', d['value'], d['ms_per_step'])" | tee -a $O/mlp.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 20 --warmup 5 --no-sweep > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
cut -d, -f1-4 $O/kernel_stats.csv | head -12
