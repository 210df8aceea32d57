#!/bin/bash
export DGT_ALLOW_OVERSUBSCRIBE=1  # ranks share the one card of the rehearsal box
# A/B of the 2- and 8-rank exchange rehearsal between this tree and _ab/ (interleaved).
set -o pipefail
export TMPDIR=/tmp DGT_BACKEND=gloo OMP_NUM_THREADS=1 DGT_EXCHANGE_TIMEOUT_S=20
mkdir -p gpurun_out
for rep in 1 2; do
  for n in 2 4 8; do
    for t in _ab .; do
      (cd $t && timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr=127.0.0.1 --master-port=$((29700+n+rep)) bench.py --gpus $n --steps 50000 --warmup 2000 --no-sweep > /tmp/abx.json 2> /tmp/abx.err) || { tail -5 /tmp/abx.err; exit 1; }
      python -c "import json; d=json.loads(open('/tmp/abx.json').read().splitlines()[-1]); print('$t', $n, d['global_steps_per_sec'], round(d['ms_per_step']*1e3,3), d['config']['exchange'], d['params_consistent_across_ranks'])" | tee -a gpurun_out/ab_xch.txt
    done
  done
done
