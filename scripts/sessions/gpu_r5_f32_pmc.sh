# round 5: PMC counters of the exact-fp32 GEMM vs hipBLASLt (one rocprofv3 pass per counter group)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r5pmc
mkdir -p $OUT
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES"
TC="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
for shape in "4096 4096 4096" "1024 1024 1024"; do
  for prod in fwd wgrad blas; do
    tag=$(echo $shape | tr ' ' x)_$prod
    timeout -s KILL 90 rocprofv3 --pmc $SQ -d $OUT/sq_$tag -o run --output-format csv -- python3 scripts/gemm_f32_one.py $shape $prod 5 > $OUT/sq_$tag.log 2>&1 || exit 1
    timeout -s KILL 90 rocprofv3 --pmc $TC -d $OUT/tc_$tag -o run --output-format csv -- python3 scripts/gemm_f32_one.py $shape $prod 5 > $OUT/tc_$tag.log 2>&1 || exit 1
  done
done
