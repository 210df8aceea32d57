#!/bin/bash
# rocprofv3 kernel traces of the MLP trainer schedules (per-kernel time + start/end for overlap).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for sch in ${SCHEDS:-serial overlap}; do
  DGT_MLP_SCHEDULE=$sch timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$sch -o run -- python bench.py --model mlp --steps 20 --warmup 5 > gpurun_out/prof_$sch.log 2>&1 || { tail -20 gpurun_out/prof_$sch.log; exit 1; }
done
find gpurun_out -name "*kernel_stats.csv" | head
