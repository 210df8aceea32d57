#!/bin/bash
# MLP kernels: GPU tests, bench, kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_mlp_gemm.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_mlp.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 > gpurun_out/bench_mlp.json 2> gpurun_out/bench_mlp.err || { tail -20 gpurun_out/bench_mlp.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_mlp.json')); print(d['value'], d['ms_per_step'], d['model_tflops'])"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mlp -o run -- python bench.py --model mlp --steps 20 --warmup 5 > gpurun_out/prof_mlp.log 2>&1 || { tail -20 gpurun_out/prof_mlp.log; exit 1; }
