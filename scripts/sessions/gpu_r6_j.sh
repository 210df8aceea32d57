#!/bin/bash
# round 6, session J: were the old "side stream loses" A/Bs of the bf16 MLP step measured with side
# streams that shared the compute stream's hardware queue (running in turn, not beside it)?  With
# side streams now measured onto another queue (accelerator.concurrent_stream): flat (default) vs
# overlap (per-layer Adam on a side stream beside backward) vs fused wgrad+Adam in line / on a side
# stream.  N = 1, no collectives, 3 interleaved fresh processes each.
set -o pipefail
O=gpurun_out/r6j
mkdir -p $O
run() {  # run <tag> <env...> -- <args>
  local tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --model mlp --steps 200 --warmup 20 --no-sweep $ARGS > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
  python -c "import json; d=json.loads([l for l in open('$O/$tag.json') if l.startswith('{')][-1]); print('$tag', d['value'], round(d['ms_per_step']*1e3,1), 'us', d['config']['impl'], d['config']['schedule'])"
}
for r in 1 2 3; do
  ARGS="--schedule flat" run flat_$r DGT_X=0 || exit 1
  ARGS="--schedule overlap" run overlap_$r DGT_X=0 || exit 1
  ARGS="--schedule flat" run fused_$r DGT_MLP_FUSED_ADAM=1 || exit 1
  ARGS="--schedule flat" run fusedside_$r DGT_MLP_FUSED_ADAM=1 DGT_MLP_WGA_SIDE=1 || exit 1
done
