#!/bin/bash
# round 6, session G: the native launcher on a CU-masked stream of its own (own hardware queue):
# trace + A/B against torch's pool stream and the Python paths
set -o pipefail
O=gpurun_out/r6g2
mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/scripts/engine_overlap_trace.py run > $GRAFT_REPO_ROOT/$O/trace.out 2> $GRAFT_REPO_ROOT/$O/trace.err \
  || { tail -20 $GRAFT_REPO_ROOT/$O/trace.err; exit 1; }
cd $GRAFT_REPO_ROOT
python3 scripts/engine_overlap_trace.py analyze $(find $O/trace -name "*kernel_trace.csv" | head -1) > $O/overlap.txt
cat $O/overlap.txt
for rep in 1 2; do
  timeout -k 10 120 python scripts/engine_overlap_bench.py --no-force 2>/dev/null | grep "^{" >> $O/ab.jsonl || exit 1
  timeout -k 10 120 python scripts/engine_overlap_bench.py 2>/dev/null | grep "^{" >> $O/ab.jsonl || exit 1
  DGT_REDUCER_THREAD=0 timeout -k 10 120 python scripts/engine_overlap_bench.py 2>/dev/null | grep "^{" >> $O/ab.jsonl || exit 1
  DGT_REDUCER_NATIVE=0 timeout -k 10 120 python scripts/engine_overlap_bench.py 2>/dev/null | grep "^{" >> $O/ab.jsonl || exit 1
done
cat $O/ab.jsonl
timeout -k 10 200 python -u -m pytest tests/test_gpu_force_collectives.py tests/test_gpu_engine.py -k "force or concurrent" -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
