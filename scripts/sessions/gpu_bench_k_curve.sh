#!/bin/bash
# The headline bench at several K (timed steps), fresh process each, warmup 5 at small K: how the
# fixed cost of one timed launch (~28 us) amortises (profiles/r2_bench_k_curve.txt).
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for k in 20 50 100 200 500 1000 5000 20000 200000; do
    w=5; [ $k -ge 5000 ] && w=2000
    timeout -k 10 120 python bench.py --steps $k --warmup $w > gpurun_out/kc.json 2> gpurun_out/kc.err || { tail -5 gpurun_out/kc.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/kc.json').read().splitlines()[-1]); print('K=$k W=$w', d['value'], round(d['ms_per_step']*1e3, 4), 'us/step', round(d['ms_per_step']*$k*1e3, 1), 'us timed')"
  done
done
