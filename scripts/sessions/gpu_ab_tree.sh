#!/bin/bash
# A/B of the headline bench between this tree and the tree in _ab/ (previous commit), interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2 3; do
  for t in _ab .; do
    (cd $t && timeout -k 10 120 python bench.py --steps 200000 --warmup 5000 > /tmp/ab.json 2> /tmp/ab.err) || { tail -5 /tmp/ab.err; exit 1; }
    python -c "import json; d=json.load(open('/tmp/ab.json')); print('$t', d['value'], round(d['ms_per_step']*1e3,4))" | tee -a gpurun_out/ab_tree.txt
  done
done
