#!/bin/bash
# round 6: HBM bytes per kernel of the bf16 MLP step (FETCH_SIZE / WRITE_SIZE, one rocprofv3 --pmc pass
# each, kernel trace for durations) -- is the flat Adam at the HBM roof, what do the GEMMs fetch.
set -o pipefail
O=gpurun_out/r6hbm
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $R/$O/$c -o run -- \
    python3 $R/bench.py --model mlp --steps 20 --warmup 5 --no-sweep --no-secondary --no-baselines > $R/$O/$c.log 2>&1 \
    || { echo "$c failed"; tail -5 $R/$O/$c.log; exit 1; }
done
cd $R && python3 scripts/hbm_summary.py $O > $O/summary.txt && cat $O/summary.txt
