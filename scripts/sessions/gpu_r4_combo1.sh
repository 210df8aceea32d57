#!/bin/bash
# Headline with the warmup tail on the bound launch path (8 fresh processes), then the fp32 GEMM
# split-target A/B and PMC passes (scripts/gpu_r4_f32b.sh).
set -o pipefail
O=gpurun_out/r4h2
mkdir -p $O
: > $O/driver8.txt
for i in 1 2 3 4 5 6 7 8; do
  DGT_BENCH_BREAKDOWN=1 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.json 2> $O/drv_$i.err || { tail -20 $O/drv_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/drv_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" | tee -a $O/driver8.txt
  grep "timed region" $O/drv_$i.err | tee -a $O/driver8.txt
done
python - <<'PY'
import statistics
v=[float(l.split()[0]) for l in open('gpurun_out/r4h2/driver8.txt') if l[0].isdigit()]
print('median', statistics.median(v), 'min', min(v), 'max', max(v))
PY
bash scripts/gpu_r4_f32b.sh
