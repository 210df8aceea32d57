#!/bin/bash
export DGT_ALLOW_OVERSUBSCRIBE=1  # ranks share the one card of the rehearsal box
# Interleaved A/B of the multi-rank exchange rehearsal (ranks sharing one GPU, gloo control plane)
# over tree copies given as arguments (e.g. _v1 .): RANKS (2 4 8), REPS (2), STEPS (30000).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp DGT_BACKEND=gloo OMP_NUM_THREADS=1 DGT_EXCHANGE_TIMEOUT_S=20
out=gpurun_out/xch_ab_trees.txt
: > $out
for rep in $(seq ${REPS:-2}); do
  for n in ${RANKS:-2 4 8}; do
    for t in "$@"; do
      (cd $t && timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr=127.0.0.1 --master-port=$((29600+n)) bench.py --gpus $n --steps ${STEPS:-30000} --warmup 2000 --no-sweep > /tmp/xab.json 2> /tmp/xab.err) || { tail -20 /tmp/xab.err; exit 1; }
      python -c "import json; d=json.loads(open('/tmp/xab.json').read().splitlines()[-1]); print('$t ranks=$n', round(d['ms_per_step']*1e3, 3), 'us/step', d['params_consistent_across_ranks'])" | tee -a $out
    done
  done
done
