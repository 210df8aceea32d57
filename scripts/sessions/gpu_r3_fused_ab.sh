#!/bin/bash
# bf16 MLP step: fused wgrad+Adam (default) vs wgrad into the bf16 gradient + one flat Adam
# (DGT_MLP_FUSED_ADAM=0), interleaved fresh processes, then one rocprofv3 kernel-stats run of each.
set -o pipefail
mkdir -p gpurun_out/fab
export TMPDIR=/tmp
for i in 1 2 3; do
  for f in 1 0; do
    DGT_MLP_FUSED_ADAM=$f timeout -k 10 300 python bench.py --model mlp --steps 50 --warmup 10 --no-sweep > gpurun_out/fab/f${f}_$i.json 2> gpurun_out/fab/f${f}_$i.err || { tail -20 gpurun_out/fab/f${f}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/fab/f${f}_$i.json')); print('fused=$f run $i', d['value'], d['ms_per_step'])"
  done
done
cd /tmp
for f in 1 0; do
  DGT_MLP_FUSED_ADAM=$f timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/fab/prof_$f -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model mlp --steps 20 --warmup 5 --no-sweep > $GRAFT_REPO_ROOT/gpurun_out/fab/prof_$f.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/fab/prof_$f.log; exit 1; }
done
ls $GRAFT_REPO_ROOT/gpurun_out/fab/prof_1
