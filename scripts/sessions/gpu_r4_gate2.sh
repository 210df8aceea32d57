#!/bin/bash
# After the 256x256 default moved to cross-phase prefetch and the bench's launch was pre-bound:
# GEMM tests, headline launch probe, 4 driver-shape benches, 3 MLP benches, PMC passes of the
# 256x256 kernels (2 vs 8 vs hipBLASLt) on the MLP wgrad and 8192^3.
set -o pipefail
O=gpurun_out/r4g2
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
echo "== pytest test_mlp_gemm"
timeout -k 10 400 python -u -m pytest tests/test_mlp_gemm.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; exit $rc; }
echo "== headline launch probe"
timeout -k 10 200 python scripts/headline_launch_probe.py > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.jsonl
echo "== driver shape x4"
for i in 1 2 3 4; do
  DGT_BENCH_BREAKDOWN=1 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.json 2> $O/drv_$i.err || { tail -20 $O/drv_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/drv_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
  grep "timed region" $O/drv_$i.err
done
echo "== MLP x3"
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['model_tflops'])"
done
echo "== PMC"
sets=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAIT_ANY"
      "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU")
run() {  # tag M N K variant mode
  local i=0
  for set in "${sets[@]}"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $set -d $R/$O/pmc/$1_$i -o run --output-format csv -- python3 $R/scripts/gemm_one.py $2 $3 $4 $5 20 $6 > $R/$O/pmc_$1_$i.log 2>&1 || { echo "$1 pass $i failed"; tail -5 $R/$O/pmc_$1_$i.log; exit 1; }
  done
}
run wgrad_v2 4096 4096 1024 2 plain
run wgrad_v8 4096 4096 1024 8 plain
run wgrad_blas 4096 4096 1024 -1 plain
run big_v8 8192 8192 8192 8 plain
run big_blas 8192 8192 8192 -1 plain
for t in wgrad_v2 wgrad_v8 wgrad_blas big_v8 big_blas; do
  echo "== $t"; python3 $R/scripts/pmc_summary.py $R/$O/pmc/${t}_*
done > $O/pmc_summary.txt
cat $O/pmc_summary.txt | head -80
echo done
