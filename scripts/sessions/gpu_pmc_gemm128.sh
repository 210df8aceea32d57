#!/bin/bash
# PMC passes (one counter group per run) on the M=1024 forward GEMM shape (128x128 4-stage 8-wave kernel).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAIT_ANY" "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $set -d $R/gpurun_out/pmc128_$i -o run --output-format csv -- python3 $R/scripts/gemm_one.py 1024 4096 4096 0 20 > $R/gpurun_out/pmc128_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc128_$i.log; exit 1; }
done
echo done
