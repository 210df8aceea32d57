#!/bin/bash
# PMC passes (one counter group per run, rocprofv3 --pmc with --kernel-trace only) on the MLP's
# M=1024 forward GEMM: this framework's default 128x128 kernel (variant 0 -> 8-wave 4-stage) vs
# hipBLASLt (torch.matmul, variant -1).  Summarised by scripts/pmc_summary.py.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
sets=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAIT_ANY"
      "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
      "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU")
for v in 0 -1; do
  i=0
  for set in "${sets[@]}"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $set -d $R/gpurun_out/pmcg_${v}_$i -o run --output-format csv -- python3 $R/scripts/gemm_one.py 1024 4096 4096 $v 20 > $R/gpurun_out/pmcg_${v}_$i.log 2>&1 || { echo "variant $v pass $i failed"; tail -5 $R/gpurun_out/pmcg_${v}_$i.log; exit 1; }
  done
done
echo done
