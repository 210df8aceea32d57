#!/bin/bash
# Interleaved A/B/... of the headline bench over several tree copies given as arguments
# (e.g. _ab _v1 _v2 .): long K (per-step cost) and the driver's K=20 / W=5 (fixed launch cost).
# REPS=n repetitions (3); KS="steps,warmup ..." shapes ("200000,5000 20,5").
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_trees.txt
trees=("$@")
: > $out
for rep in $(seq ${REPS:-3}); do
  for t in "${trees[@]}"; do
    for k in ${KS:-200000,5000 20,5}; do
      k=${k/,/ }
      set -- $k
      (cd $t && DGT_BENCH_BREAKDOWN=1 timeout -k 10 120 python bench.py --steps $1 --warmup $2 > /tmp/ab.json 2> /tmp/ab.err) || { tail -5 /tmp/ab.err; exit 1; }
      python -c "import json; d=json.loads([l for l in open('/tmp/ab.json') if l.startswith('{')][-1]); print('$t', 'K=$1', d['value'], round(d['ms_per_step']*1e3,4), 'us/step')" | tee -a $out
      grep -h "timed region" /tmp/ab.err >> $out || true
    done
  done
done
