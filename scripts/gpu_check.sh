#!/bin/bash
# One GPU session: build, numerics tests, benches, kernel profile.  Every GPU step is bounded.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== build"; timeout -k 10 300 python tools/build_ext.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
echo "== pytest gpu"; timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench fused"; timeout -k 10 300 python bench.py --steps 100000 --warmup 5000 > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err || { tail -20 gpurun_out/bench_fused.err; exit 1; }
cat gpurun_out/bench_fused.json
echo "== bench stepwise"; timeout -k 10 300 python bench.py --impl stepwise --steps 3000 --warmup 300 > gpurun_out/bench_stepwise.json 2> gpurun_out/bench_stepwise.err || { tail -20 gpurun_out/bench_stepwise.err; exit 1; }
cat gpurun_out/bench_stepwise.json
echo "== bench engine"; timeout -k 10 300 python bench.py --impl engine --steps 2000 --warmup 200 > gpurun_out/bench_engine.json 2> gpurun_out/bench_engine.err || { tail -20 gpurun_out/bench_engine.err; exit 1; }
cat gpurun_out/bench_engine.json
echo "== rocprof"; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20000 --warmup 500 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1; echo "rocprof rc=$?"
find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*stats*" | head
