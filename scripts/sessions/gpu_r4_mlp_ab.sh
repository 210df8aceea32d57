#!/bin/bash
# bf16 MLP step: register-prefetch GEMMs on the forward (variant 7) and/or the dgrad (variant 6)
# only, through the trainer's per-product knobs (DGT_GEMM_VARIANT would also move the wgrad off the
# 256x256 kernel), interleaved; then a rocprofv3 --stats session of the best-guess configuration.
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
: > $O/mlp_ab.txt
for rep in 1 2 3; do
for cfg in "0 0" "7 0" "0 6" "7 6"; do
  set -- $cfg
  DGT_MLP_FWD_VARIANT=$1 DGT_MLP_DGRAD_VARIANT=$2 timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print('fwd $1 dgrad $2', d['value'], d['ms_per_step'], d['model_tflops'])" | tee -a $O/mlp_ab.txt
done
done
echo "== rocprofv3 --stats, fwd 7 dgrad 6"
export TMPDIR=/tmp
DGT_MLP_FWD_VARIANT=7 DGT_MLP_DGRAD_VARIANT=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --model mlp --steps 50 --warmup 10 --no-sweep > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/mlp_rp_kernel_stats.csv
cut -d, -f1-4 $O/mlp_rp_kernel_stats.csv | head -12
