#!/bin/bash
# round 6, session D: the native launcher's side stream at high priority (its own hardware queue)
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/scripts/engine_overlap_trace.py run > $GRAFT_REPO_ROOT/$O/trace.out 2> $GRAFT_REPO_ROOT/$O/trace.err \
  || { tail -20 $GRAFT_REPO_ROOT/$O/trace.err; exit 1; }
cd $GRAFT_REPO_ROOT
grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl" $O/trace.out
python3 scripts/engine_overlap_trace.py analyze $(find $O/trace -name "*kernel_trace.csv" | head -1) > $O/overlap.txt
cat $O/overlap.txt
timeout -k 10 120 python -u -m pytest tests/test_gpu_force_collectives.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
