#!/bin/bash
# bf16 MLP step: the flat Adam's bf16 weight copy stored cacheably (DGT_ADAM_LP_KEEP=1: it stays in
# the Infinity Cache for the next forward's GEMMs) or streamed (0, default), x the 128x128 GEMM form
# (DGT_GEMM_VARIANT=0: front-loaded reads, 5: software-pipelined reads); interleaved fresh processes,
# then rocprofv3 kernel stats of the two extreme arms.
set -o pipefail
mkdir -p gpurun_out/lpk
export TMPDIR=/tmp
for i in 1 2 3; do
  for k in 0 1; do
    for v in 0 5; do
      DGT_ADAM_LP_KEEP=$k DGT_GEMM_VARIANT=$v timeout -k 10 300 python bench.py --model mlp --steps 100 --warmup 10 --no-sweep > gpurun_out/lpk/k${k}v${v}_$i.json 2> gpurun_out/lpk/k${k}v${v}_$i.err || { tail -20 gpurun_out/lpk/k${k}v${v}_$i.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/lpk/k${k}v${v}_$i.json')); print('lp_keep=$k variant=$v run $i', d['value'], d['ms_per_step'])"
    done
  done
done
cd /tmp
for kv in "0 0" "1 5"; do
  set -- $kv
  DGT_ADAM_LP_KEEP=$1 DGT_GEMM_VARIANT=$2 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/lpk/prof_k$1v$2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model mlp --steps 20 --warmup 5 --no-sweep > $GRAFT_REPO_ROOT/gpurun_out/lpk/prof_k$1v$2.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/lpk/prof_k$1v$2.log; exit 1; }
done
