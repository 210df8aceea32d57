#!/bin/bash
# PMC passes (one counter group per run, --kernel-trace only) on the round-3 kernels: the MLP dgrad
# (1024 x 4096 x 4096, [K,N] W, mask + C^T + column sums) on SP (variant 5, the shape rule's choice)
# and FR (variant 3) vs hipBLASLt's plain g @ W, and the wgrad 4096 x 4096 x 1024 on the one-barrier
# 256x256 kernel vs hipBLASLt.  Summaries: scripts/pmc_summary.py.
set -o pipefail
mkdir -p gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
sets=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAIT_ANY"
      "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU")
run() {  # tag M N K variant mode
  local i=0
  for set in "${sets[@]}"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $set -d $R/gpurun_out/pmc2/$1_$i -o run --output-format csv -- python3 $R/scripts/gemm_one.py $2 $3 $4 $5 20 $6 > $R/gpurun_out/pmc2/$1_$i.log 2>&1 || { echo "$1 pass $i failed"; tail -5 $R/gpurun_out/pmc2/$1_$i.log; exit 1; }
  done
}
run dgrad_sp 1024 4096 4096 5 dgrad
run dgrad_fr 1024 4096 4096 3 dgrad
run dgrad_blas 1024 4096 4096 -1 dgrad
run wgrad_256 4096 4096 1024 2 plain
run wgrad_blas 4096 4096 1024 -1 plain
for t in dgrad_sp dgrad_fr dgrad_blas wgrad_256 wgrad_blas; do
  echo "== $t"; python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc2/${t}_*
done > $R/gpurun_out/pmc2/summary.txt
echo done
