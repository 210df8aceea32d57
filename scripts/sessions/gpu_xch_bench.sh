#!/bin/bash
export DGT_ALLOW_OVERSUBSCRIBE=1  # ranks share the one card of the rehearsal box
# Exchange rehearsal benches on one GPU (gloo control plane): 2, 4 and 8 ranks through the fused
# kernel; at 4 and 8 ranks the ZeRO-0 one-shot and ZeRO-1 exchanges in both line formats
# (DGT_XCH_LINE=ll3 / ll2; --zero-stage 0 / 1), REPS times interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp DGT_BACKEND=gloo OMP_NUM_THREADS=1 DGT_EXCHANGE_TIMEOUT_S=20
run() {  # run <ranks> <line> <zero stage> <tag>
  local n=$1 mode=$2 zero=$3 tag=$4
  DGT_XCH_LINE=$mode timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr=127.0.0.1 --master-port=$((29600+n)) bench.py --gpus $n --steps ${STEPS:-50000} --warmup 2000 --no-sweep --zero-stage $zero > gpurun_out/xch_$tag.json 2> gpurun_out/xch_$tag.err || { tail -20 gpurun_out/xch_$tag.err; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/xch_$tag.json').read().splitlines()[-1]); print($n, '$mode', 'zero$zero', d['global_steps_per_sec'], round(d['ms_per_step']*1e3, 3), 'us/step', d['config']['exchange'], d['params_consistent_across_ranks'])"
}
run 2 auto 0 2 || exit 1
for r in $(seq 1 ${REPS:-1}); do
  for n in ${RANKS:-4 8}; do
    for mode in ll3 ll2; do
      for zero in 0 1; do
        run $n $mode $zero ${n}_${mode}_z${zero}_$r || exit 1
      done
    done
  done
done
