#!/bin/bash
# round 6, first GPU session: the new tests (engine fuzz, shipped-config fast paths, dropout RNG,
# in-place check, engine MLP forced collectives) + the full GPU suite, the bench with its same-run
# torch baselines, the kernel trace of the engine's per-layer bucket launches (overlap proof) and
# the whole-step graph's process-to-process spread (4 fresh processes unpinned, 4 pinned).
set -o pipefail
mkdir -p gpurun_out/r6a
export TMPDIR=/tmp
O=gpurun_out/r6a
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/scripts/engine_overlap_trace.py run > $GRAFT_REPO_ROOT/$O/trace.out 2> $GRAFT_REPO_ROOT/$O/trace.err \
  || { tail -20 $GRAFT_REPO_ROOT/$O/trace.err; exit 1; }
cd $GRAFT_REPO_ROOT
cat $O/trace.out
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/engine_overlap_trace.py analyze $f > $O/overlap.txt && tail -40 $O/overlap.txt
for i in 1 2 3 4; do
  timeout -k 10 120 python scripts/graph_variance_probe.py >> $O/variance.jsonl 2>> $O/variance.err || exit 1
done
cpu=$(python -c "import os; print(sorted(os.sched_getaffinity(0))[2])")
for i in 1 2 3 4; do
  timeout -k 10 120 python scripts/graph_variance_probe.py --pin $cpu >> $O/variance.jsonl 2>> $O/variance.err || exit 1
done
cat $O/variance.jsonl
exit $rc
