#!/bin/bash
export DGT_ALLOW_OVERSUBSCRIBE=1  # ranks share the one card of the rehearsal box
# Exchange rehearsal benches on one GPU (gloo control plane): 2, 4 and 8 ranks through the fused
# kernel; at 4 and 8 ranks both protocols (DGT_XCH=oneshot / twoshot), REPS times interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp DGT_BACKEND=gloo OMP_NUM_THREADS=1 DGT_EXCHANGE_TIMEOUT_S=20
run() {  # run <ranks> <mode> <tag>
  local n=$1 mode=$2 tag=$3
  DGT_XCH=$mode timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr=127.0.0.1 --master-port=$((29600+n)) bench.py --gpus $n --steps ${STEPS:-50000} --warmup 2000 --no-sweep > gpurun_out/xch_$tag.json 2> gpurun_out/xch_$tag.err || { tail -20 gpurun_out/xch_$tag.err; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/xch_$tag.json').read().splitlines()[-1]); print($n, '$mode', d['global_steps_per_sec'], round(d['ms_per_step']*1e3, 3), 'us/step', d['config']['exchange'], d['params_consistent_across_ranks'])"
}
run 2 auto 2 || exit 1
for r in $(seq 1 ${REPS:-1}); do
  for n in ${RANKS:-4 8}; do
    for mode in oneshot twoshot; do
      run $n $mode ${n}_${mode}_$r || exit 1
    done
  done
done
