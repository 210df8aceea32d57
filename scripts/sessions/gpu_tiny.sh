#!/bin/bash
# Fused tiny-kernel session: numerics, headline bench, stamped section breakdown.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest tiny"; timeout -k 10 600 python -m pytest tests/test_gpu_tiny_mlp.py -x -q -m gpu > gpurun_out/pytest_tiny.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_tiny.log; [ $rc -eq 0 ] || exit $rc
echo "== bench fused"; timeout -k 10 300 python bench.py --steps 100000 --warmup 5000 > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err || { tail -20 gpurun_out/bench_fused.err; exit 1; }
cat gpurun_out/bench_fused.json
echo "== stamps"; timeout -k 10 120 ./build/bin/tiny_stamps > gpurun_out/tiny_stamps.txt 2>&1; rc=$?; cat gpurun_out/tiny_stamps.txt; exit $rc
