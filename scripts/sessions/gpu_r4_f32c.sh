#!/bin/bash
# fp32 GEMM after the fragment read-ahead, interior fast path and auto split target: numerics tests,
# microbench vs hipBLASLt, fp32 engine MLP x2, PMC of the 4096^3 forward.
set -o pipefail
O=gpurun_out/r4f3
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gemm_f32.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/bench_gemm_f32.py > $O/gemm.jsonl 2> $O/gemm.err || { tail -20 $O/gemm.err; exit 1; }
cat $O/gemm.jsonl
for i in 1 2; do
  timeout -k 10 300 python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 50 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print('fp32 engine MLP', d['value'], d['ms_per_step'])"
done
sets=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAIT_ANY"
      "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU")
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $set -d $R/$O/pmc/fwd4k_$i -o run --output-format csv -- python3 $R/scripts/gemm_f32_one.py 4096 4096 4096 fwd 10 > $R/$O/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/$O/pmc_$i.log; exit 1; }
done
python3 $R/scripts/pmc_summary.py $R/$O/pmc/fwd4k_* > $O/pmc_summary.txt
grep -A16 "gemm_f32_kernel" $O/pmc_summary.txt | head -20
