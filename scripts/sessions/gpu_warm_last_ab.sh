#!/bin/bash
# bench.py at the driver's shape with the last warmup step held back until right before the opening
# sync (DGT_BENCH_WARM_LAST=1, default) vs run with the others (0); interleaved fresh processes.
set -o pipefail
mkdir -p gpurun_out
for r in $(seq ${REPS:-5}); do
  for v in 0 1; do
    DGT_BENCH_WARM_LAST=$v DGT_BENCH_BREAKDOWN=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/wl.json 2> gpurun_out/wl.err || { tail -5 gpurun_out/wl.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/wl.json').read().splitlines()[-1]); print('warm_last=$v', d['value'], round(d['ms_per_step'] * 1e3, 3), 'us/step', d['mean_loss'])"
    grep -h "timed region" gpurun_out/wl.err
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_multiproc.py -k "bench" 2>&1 | tail -1
