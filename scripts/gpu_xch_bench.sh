#!/bin/bash
# Exchange rehearsal benches on one GPU (gloo control plane): 2 and 8 ranks through the fused kernel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp DGT_BACKEND=gloo OMP_NUM_THREADS=1 DGT_EXCHANGE_TIMEOUT_S=20
for n in 2 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr=127.0.0.1 --master-port=$((29600+n)) bench.py --gpus $n --steps ${STEPS:-50000} --warmup 2000 --no-sweep > gpurun_out/xch_$n.json 2> gpurun_out/xch_$n.err || { tail -20 gpurun_out/xch_$n.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/xch_$n.json').read().splitlines()[-1]); print($n, d['global_steps_per_sec'], d['ms_per_step']*1e3, 'us/step', d['config']['exchange'], d['params_consistent_across_ranks'])"
done
