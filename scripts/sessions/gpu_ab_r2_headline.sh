#!/bin/bash
# Headline A/B on one box: the round-2 tree (build/abr2, built from commit 96c0023) against the
# current tree, interleaved, fresh process per run: default shape and the driver's K = 20 shape.
set -o pipefail
mkdir -p gpurun_out/abh
export TMPDIR=/tmp
for i in 1 2 3; do
  for t in r2 r3; do
    d=$([ $t = r2 ] && echo build/abr2 || echo .)
    (cd $d && timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-sweep) > gpurun_out/abh/${t}_drv_$i.json 2> gpurun_out/abh/${t}_drv_$i.err || { tail -5 gpurun_out/abh/${t}_drv_$i.err; exit 1; }
    (cd $d && timeout -k 10 200 python bench.py --no-sweep) > gpurun_out/abh/${t}_def_$i.json 2> gpurun_out/abh/${t}_def_$i.err || { tail -5 gpurun_out/abh/${t}_def_$i.err; exit 1; }
    python -c "import json; a=json.load(open('gpurun_out/abh/${t}_drv_$i.json')); b=json.load(open('gpurun_out/abh/${t}_def_$i.json')); print('$t run $i driver', a['value'], 'default', b['value'], b['ms_per_step'])"
  done
done
