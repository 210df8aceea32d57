#!/bin/bash
# Round-3 exchange validation on one MI355X: single-rank fused kernel + ZeRO-1 config, every
# multi-rank rehearsal (LL3 / LL2 line formats, ZeRO-1 exchange, stress self-test, run-time
# fallback), then the headline bench at the driver's shape.
set -o pipefail
mkdir -p gpurun_out/r3a
export TMPDIR=/tmp DGT_QUIET=1
P="python -u -m pytest -v --timeout 600 --timeout-method thread"
timeout -k 10 600 $P tests/test_gpu_tiny_mlp.py tests/test_gpu_train.py tests/test_gpu_engine.py tests/test_mlp_gemm.py > gpurun_out/r3a/pytest_single.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r3a/pytest_single.log | tail -30; exit 1; }
tail -2 gpurun_out/r3a/pytest_single.log
timeout -k 10 900 $P tests/test_gpu_multiproc.py -k "${MP_K:-fallback or strict or stress or zero1 or every_shape or many_ranks}" > gpurun_out/r3a/pytest_multi.log 2>&1 || { tail -60 gpurun_out/r3a/pytest_multi.log; exit 1; }
tail -2 gpurun_out/r3a/pytest_multi.log
for i in 1 2 3; do
  DGT_BENCH_BREAKDOWN=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r3a/bench_$i.json 2> gpurun_out/r3a/bench_$i.err || { tail -20 gpurun_out/r3a/bench_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r3a/bench_$i.json')); print(d['value'], d['ms_per_step'])"
done
echo done
