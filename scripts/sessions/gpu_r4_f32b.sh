#!/bin/bash
# fp32 GEMM: split-K block target A/B (DGT_F32_MIN_BLOCKS 256 / 512 / 1024) on the small shapes and
# the fp32 engine MLP, then PMC passes of the 4096^3 forward vs hipBLASLt.
set -o pipefail
O=gpurun_out/r4f2
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for mb in 256 512 1024; do
  echo "== min_blocks $mb"
  DGT_F32_MIN_BLOCKS=$mb timeout -k 10 200 python scripts/bench_gemm_f32.py 1024x1024x1024 1000x1000x1000 256x4096x4096 1024x4096x4096 > $O/gemm_mb$mb.jsonl 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
  cat $O/gemm_mb$mb.jsonl
  DGT_F32_MIN_BLOCKS=$mb timeout -k 10 300 python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 50 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print('fp32 engine MLP', d['value'], d['ms_per_step'])"
done
sets=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAIT_ANY"
      "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU")
run() {
  local i=0
  for set in "${sets[@]}"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $set -d $R/$O/pmc/$1_$i -o run --output-format csv -- python3 $R/scripts/gemm_f32_one.py $2 $3 $4 $5 10 > $R/$O/pmc_$1_$i.log 2>&1 || { echo "$1 pass $i failed"; tail -5 $R/$O/pmc_$1_$i.log; exit 1; }
  done
}
run fwd4k 4096 4096 4096 fwd
run blas4k 4096 4096 4096 blas
run fwd1k 1024 1024 1024 fwd
run blas1k 1024 1024 1024 blas
for t in fwd4k blas4k fwd1k blas1k; do
  echo "== $t"; python3 $R/scripts/pmc_summary.py $R/$O/pmc/${t}_*
done > $O/pmc_summary.txt
grep -E "^==|^void|^Cijk|MFMA_BUSY|SQ_BUSY|SQ_WAVES|SQ_WAVE_CYCLES|WAIT_ANY|INSTS_VALU|LDS_BANK" $O/pmc_summary.txt | head -80
