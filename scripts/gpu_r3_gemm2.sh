#!/bin/bash
# Round-3 GEMM A/B #2: variant 3 (front-loaded reads) vs 5 (same, one barrier per two K-tiles) vs
# 4 (round-2 default) on the M = 1024 products and inside the MLP step (interleaved runs).
set -o pipefail
mkdir -p gpurun_out/r3g3
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_mlp_gemm.py > gpurun_out/r3g3/pytest_gemm.log 2>&1 || { tail -30 gpurun_out/r3g3/pytest_gemm.log; exit 1; }
tail -1 gpurun_out/r3g3/pytest_gemm.log
CHECK_VARIANT=5 VARIANTS=4,3,5 timeout -k 10 300 python scripts/bench_gemm_m1024.py > gpurun_out/r3g3/m1024.jsonl 2> gpurun_out/r3g3/m1024.err || { tail -20 gpurun_out/r3g3/m1024.err; exit 1; }
cat gpurun_out/r3g3/m1024.jsonl
for i in 1 2; do
  for v in 4 3 5; do
    DGT_GEMM_VARIANT=$v timeout -k 10 300 python bench.py --model mlp --steps 50 --warmup 10 > gpurun_out/r3g3/mlp_v${v}_$i.json 2> gpurun_out/r3g3/mlp_v${v}_$i.err || { tail -20 gpurun_out/r3g3/mlp_v${v}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r3g3/mlp_v${v}_$i.json')); print('mlp variant $v run $i', d['value'], d['ms_per_step'])"
  done
done

cd /tmp
R=$GRAFT_REPO_ROOT
for v in 3 5 -1; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAIT_ANY -d $R/gpurun_out/r3g3/pmc_${v} -o run --output-format csv -- python3 $R/scripts/gemm_one.py 1024 4096 4096 $v 20 fwd > $R/gpurun_out/r3g3/pmc_${v}.log 2>&1 || { echo "pmc $v failed"; tail -5 $R/gpurun_out/r3g3/pmc_${v}.log; exit 1; }
done
echo pmc done
