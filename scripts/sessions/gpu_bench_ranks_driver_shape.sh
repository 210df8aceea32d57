#!/bin/bash
export DGT_ALLOW_OVERSUBSCRIBE=1  # ranks share the one card of the rehearsal box
# The driver's bench shape (--steps 20 --warmup 5) with 2 and 8 ranks sharing one GPU, closing the
# timed region with the IPC device barrier (default) vs the process-group barrier
# (DGT_BENCH_PG_BARRIER=1), REPS interleaved fresh-process runs each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp DGT_BACKEND=${DGT_BACKEND:-gloo} OMP_NUM_THREADS=1 DGT_EXCHANGE_TIMEOUT_S=20 DGT_BENCH_BREAKDOWN=1
for r in $(seq 1 ${REPS:-3}); do
  for n in ${RANKS:-2 8}; do
    for pg in ${PGS:-"" 1}; do
      tag=${n}_${pg:-dev}_$r
      DGT_BENCH_PG_BARRIER=$pg timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr=127.0.0.1 --master-port=$((29700+n)) bench.py --gpus $n --steps 20 --warmup 5 --no-sweep > gpurun_out/ds_$tag.json 2> gpurun_out/ds_$tag.err || { tail -20 gpurun_out/ds_$tag.err; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/ds_$tag.json').read().splitlines()[-1]); print('ranks=$n', d['config']['closing_barrier'], d['value'], round(d['ms_per_step']*1e3, 2), 'us/step')"
      grep "timed region" gpurun_out/ds_$tag.err | head -1
    done
  done
done
