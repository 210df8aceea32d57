#!/bin/bash
# round 6, session C: the native bucket launcher (csrc/bucket_launcher.cpp): forced-collective engine
# paths bit-identical, host cost per bucket, the overlap trace of the bf16 engine MLP.
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_force_collectives.py tests/test_gpu_engine.py tests/test_gpu_engine_fuzz.py \
  -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
if [ $rc -ne 0 ]; then grep -B5 -A30 "force_collectives.*FAILED\|Error" $O/pytest.log | head -60; exit $rc; fi
timeout -k 10 120 python scripts/reducer_host_cost.py > $O/host_cost.json 2> $O/host_cost.err || { tail -20 $O/host_cost.err; exit 1; }
cat $O/host_cost.json
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/scripts/engine_overlap_trace.py run > $GRAFT_REPO_ROOT/$O/trace.out 2> $GRAFT_REPO_ROOT/$O/trace.err \
  || { tail -20 $GRAFT_REPO_ROOT/$O/trace.err; exit 1; }
cd $GRAFT_REPO_ROOT
grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl" $O/trace.out
python3 scripts/engine_overlap_trace.py analyze $(find $O/trace -name "*kernel_trace.csv" | head -1) > $O/overlap.txt
cat $O/overlap.txt
