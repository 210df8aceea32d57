#!/bin/bash
# round 6, session B: the fixed whole-step graph (step counter / lr sync, stale bucket), the reducer's
# launcher thread (host cost per bucket launch, overlap trace), engine host-thread pinning (4 fresh
# processes pinned by the config, 2 unpinned), the driver-shape bench with its baselines.
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine_fuzz.py tests/test_gpu_force_collectives.py \
  tests/test_gpu_engine.py -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python scripts/reducer_host_cost.py > $O/host_cost.json 2> $O/host_cost.err || { tail -20 $O/host_cost.err; exit 1; }
cat $O/host_cost.json
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/scripts/engine_overlap_trace.py run > $GRAFT_REPO_ROOT/$O/trace.out 2> $GRAFT_REPO_ROOT/$O/trace.err \
  || { tail -20 $GRAFT_REPO_ROOT/$O/trace.err; exit 1; }
cd $GRAFT_REPO_ROOT
cat $O/trace.out
python3 scripts/engine_overlap_trace.py analyze $(find $O/trace -name "*kernel_trace.csv" | head -1) > $O/overlap.txt
tail -12 $O/overlap.txt
for i in 1 2 3 4; do
  timeout -k 10 120 python scripts/graph_variance_probe.py >> $O/variance.jsonl 2>> $O/variance.err || exit 1
done
for i in 1 2; do
  timeout -k 10 120 python scripts/graph_variance_probe.py --unpinned >> $O/variance.jsonl 2>> $O/variance.err || exit 1
done
cat $O/variance.jsonl
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -c 1500 $O/bench.json
exit $rc
