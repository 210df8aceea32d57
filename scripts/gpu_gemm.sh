#!/bin/bash
# GEMM session: numerics for both tile kernels, then the GEMM micro-benchmark and the MLP bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest gemm"; timeout -k 10 600 python -m pytest tests/test_mlp_gemm.py -x -q -m gpu > gpurun_out/pytest_gemm.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
echo "== gemm bench"; timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.jsonl || exit 1
cat gpurun_out/bench_gemm.jsonl
echo "== mlp bench"; timeout -k 10 300 python bench.py --model mlp --steps 30 --warmup 5 --no-sweep > gpurun_out/bench_mlp.json 2> gpurun_out/bench_mlp.err || { tail -20 gpurun_out/bench_mlp.err; exit 1; }
cat gpurun_out/bench_mlp.json
echo "== rocprof mlp"; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_mlp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model mlp --steps 10 --warmup 2 --no-sweep > $GRAFT_REPO_ROOT/gpurun_out/prof_mlp.log 2>&1; echo "rocprof rc=$?"
