#!/bin/bash
# One GPU session: GPU test suite, smoke(), headline bench (1 GPU), bench-size MLP bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "== bench default"
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
echo "== bench mlp"
timeout -k 10 300 python bench.py --model mlp --steps 50 --warmup 5 > gpurun_out/bench_mlp.json 2> gpurun_out/bench_mlp.err || { tail -20 gpurun_out/bench_mlp.err; exit 1; }
cat gpurun_out/bench_mlp.json
