#!/bin/bash
# A/B of the bench-size MLP between this tree and the tree in _ab/ (previous commit), interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2 3; do
  for t in _ab .; do
    (cd $t && timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 --no-sweep > /tmp/ab.json 2> /tmp/ab.err) || { tail -5 /tmp/ab.err; exit 1; }
    python -c "import json; d=json.load(open('/tmp/ab.json')); print('$t', d['value'], d['ms_per_step'])" | tee -a gpurun_out/ab_mlp_tree.txt
  done
done
