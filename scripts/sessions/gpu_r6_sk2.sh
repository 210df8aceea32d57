#!/bin/bash
# round 6: why the split-K kernel's loop is slow -- kernel-trace timing of the loop alone / the
# epilogue without the meeting / the full kernel, and one SQ counter pass each for v3 and v9.
set -o pipefail
O=gpurun_out/r6sk2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
for xs in 1 3 5 0 2; do
  DGT_GEMM_SK_XS=$xs timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/t_xs$xs -o run -- \
    python3 $R/scripts/gemm_one.py 1024 4096 4096 9 30 fwd > $R/$O/t_xs$xs.log 2>&1 || { echo "xs $xs failed"; tail -5 $R/$O/t_xs$xs.log; exit 1; }
  echo "xs=$xs"; grep -h "gemm_nt_sk" $(find $R/$O/t_xs$xs -name "*kernel_stats.csv") | cut -d, -f1-4
done
for v in 3 9; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAIT_ANY \
    -d $R/$O/pmc_v$v -o run --output-format csv -- python3 $R/scripts/gemm_one.py 1024 4096 4096 $v 20 fwd > $R/$O/pmc_v$v.log 2>&1 || { echo "pmc v$v failed"; tail -5 $R/$O/pmc_v$v.log; exit 1; }
done
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_MFMA SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY \
  -d $R/$O/pmc2_v9 -o run --output-format csv -- python3 $R/scripts/gemm_one.py 1024 4096 4096 9 20 fwd > $R/$O/pmc2_v9.log 2>&1 || { echo "pmc2 failed"; tail -5 $R/$O/pmc2_v9.log; }
cd $R && python3 scripts/pmc_summary.py $O/pmc_v3 $O/pmc_v9 $O/pmc2_v9 2>&1 | head -80
