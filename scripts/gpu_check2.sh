#!/bin/bash
# MLP-path GPU session: full numerics suite, smoke, bench-size MLP bench + kernel profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest gpu"; timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
echo "== gemm bench"; timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.jsonl || exit 1
cat gpurun_out/bench_gemm.jsonl
echo "== mlp bench"; timeout -k 10 300 python bench.py --model mlp --steps 30 --warmup 5 --no-sweep > gpurun_out/bench_mlp.json 2> gpurun_out/bench_mlp.err || { tail -20 gpurun_out/bench_mlp.err; exit 1; }
cat gpurun_out/bench_mlp.json
echo "== bench fused"; timeout -k 10 300 python bench.py --steps 100000 --warmup 5000 > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err || { tail -20 gpurun_out/bench_fused.err; exit 1; }
cat gpurun_out/bench_fused.json
echo "== rocprof mlp"; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_mlp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model mlp --steps 10 --warmup 2 --no-sweep > $GRAFT_REPO_ROOT/gpurun_out/prof_mlp.log 2>&1; echo "rocprof rc=$?"
