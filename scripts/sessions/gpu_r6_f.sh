#!/bin/bash
# round 6, session F: full GPU suite after the native bucket launcher; its overlap trace and host cost.
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/scripts/engine_overlap_trace.py run > $GRAFT_REPO_ROOT/$O/trace.out 2> $GRAFT_REPO_ROOT/$O/trace.err \
  || { tail -20 $GRAFT_REPO_ROOT/$O/trace.err; exit 1; }
cd $GRAFT_REPO_ROOT
grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl" $O/trace.out
python3 scripts/engine_overlap_trace.py analyze $(find $O/trace -name "*kernel_trace.csv" | head -1) > $O/overlap.txt
tail -9 $O/overlap.txt
timeout -k 10 120 python scripts/reducer_host_cost.py 2>/dev/null | grep "^{" > $O/host_cost.json; cat $O/host_cost.json
exit $rc
