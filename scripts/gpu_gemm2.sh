#!/bin/bash
# GEMM session 2: numerics, micro-benchmark, MLP bench, and a PMC counter profile of both tiles.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest gemm"; timeout -k 10 600 python -m pytest tests/test_mlp_gemm.py -x -q -m gpu > gpurun_out/pytest_gemm.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
echo "== gemm bench"; timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.jsonl || exit 1
cat gpurun_out/bench_gemm.jsonl
echo "== mlp bench"; timeout -k 10 300 python bench.py --model mlp --steps 30 --warmup 5 --no-sweep > gpurun_out/bench_mlp.json 2> gpurun_out/bench_mlp.err || { tail -20 gpurun_out/bench_mlp.err; exit 1; }
cut -c1-300 gpurun_out/bench_mlp.json
echo "== pmc"; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES -d $GRAFT_REPO_ROOT/gpurun_out/pmc_gemm -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/gemm_one.py 4096 4096 4096 2 5 > $GRAFT_REPO_ROOT/gpurun_out/pmc_gemm.log 2>&1; echo "pmc rc=$?"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/pmc_gemm.log
