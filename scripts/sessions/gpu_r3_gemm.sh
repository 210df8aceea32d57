#!/bin/bash
# Round-3 GEMM session: M = 1024 products (fwd / dgrad / wgrad) hot and cold for the default 8-wave
# kernel (v4), its front-loaded-reads form (v3) and hipBLASLt; the MLP step with each; PMC passes
# (fused forward epilogue) for v4 / v3 / hipBLASLt.  Outputs under gpurun_out/r3g/.
set -o pipefail
mkdir -p gpurun_out/r3g
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
VARIANTS=4,3 WGRAD_VARIANTS=4,3,2 timeout -k 10 300 python scripts/bench_gemm_m1024.py > gpurun_out/r3g/m1024.jsonl 2> gpurun_out/r3g/m1024.err || { tail -20 gpurun_out/r3g/m1024.err; exit 1; }
cat gpurun_out/r3g/m1024.jsonl
for i in 1 2; do
  for v in 0 3; do
    DGT_GEMM_VARIANT=$v timeout -k 10 300 python bench.py --model mlp --steps 50 --warmup 10 > gpurun_out/r3g/mlp_v${v}_$i.json 2> gpurun_out/r3g/mlp_v${v}_$i.err || { tail -20 gpurun_out/r3g/mlp_v${v}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r3g/mlp_v${v}_$i.json')); print('mlp variant $v run $i', d['value'], d['ms_per_step'])"
  done
done
cd /tmp
sets=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAIT_ANY"
      "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU")
for v in 4 3 -1; do
  i=0
  for set in "${sets[@]}"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $set -d $R/gpurun_out/r3g/pmc_${v}_$i -o run --output-format csv -- python3 $R/scripts/gemm_one.py 1024 4096 4096 $v 20 fwd > $R/gpurun_out/r3g/pmc_${v}_$i.log 2>&1 || { echo "variant $v pass $i failed"; tail -5 $R/gpurun_out/r3g/pmc_${v}_$i.log; exit 1; }
  done
done
echo done
