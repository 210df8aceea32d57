#!/bin/bash
export DGT_ALLOW_OVERSUBSCRIBE=1  # ranks share the one card of the rehearsal box
# DGT_BENCH_WARM_LAST=0/1 at the driver's shape with RANKS ranks sharing one GPU (gloo control plane,
# IPC device barriers), interleaved fresh launches, REPS each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp DGT_BACKEND=${DGT_BACKEND:-gloo} OMP_NUM_THREADS=1 DGT_EXCHANGE_TIMEOUT_S=20 DGT_BENCH_BREAKDOWN=1
for r in $(seq 1 ${REPS:-3}); do
  for n in ${RANKS:-2}; do
    for v in 0 1; do
      tag=${n}_${v}_$r
      DGT_BENCH_WARM_LAST=$v timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr=127.0.0.1 --master-port=$((29700+n)) bench.py --gpus $n --steps 20 --warmup 5 --no-sweep > gpurun_out/wr_$tag.json 2> gpurun_out/wr_$tag.err || { tail -20 gpurun_out/wr_$tag.err; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/wr_$tag.json').read().splitlines()[-1]); print('ranks=$n warm_last=$v', d['value'], round(d['ms_per_step']*1e3, 2), 'us/step', d['params_consistent_across_ranks'])"
    done
  done
done
