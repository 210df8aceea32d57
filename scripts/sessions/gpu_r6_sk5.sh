#!/bin/bash
# round 6: the epilogue bias prefetch (every staged-epilogue GEMM) A/B against the previous commit's
# extension (build/variants/head) in the bf16 MLP step, alternating processes; split-K (per-phase
# meeting) timing and diagnostics once more; the SK tests.
set -o pipefail
O=gpurun_out/r6sk5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_sk.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python scripts/bench_gemm_sk.py > $O/gemm_xs1.jsonl 2>&1 || { tail -20 $O/gemm_xs1.jsonl; exit 1; }
grep -v amdgpu.ids $O/gemm_xs1.jsonl
DGT_EXT_LIB=build/variants/head/_C.so timeout -k 10 200 python scripts/bench_gemm_m1024.py > $O/gemm_head.jsonl 2>&1 || { tail -20 $O/gemm_head.jsonl; exit 1; }
timeout -k 10 200 python scripts/bench_gemm_m1024.py > $O/gemm_new.jsonl 2>&1 || { tail -20 $O/gemm_new.jsonl; exit 1; }
echo head; grep arm $O/gemm_head.jsonl; echo new; grep arm $O/gemm_new.jsonl
R=$GRAFT_REPO_ROOT
cd /tmp
for xs in 1 3 5; do
  DGT_GEMM_SK_XS=$xs timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/t_xs$xs -o run -- \
    python3 $R/scripts/gemm_one.py 1024 4096 4096 9 30 fwd > $R/$O/t_xs$xs.log 2>&1 || { echo "xs $xs failed"; tail -5 $R/$O/t_xs$xs.log; exit 1; }
  echo "xs=$xs $(grep -h gemm_nt_sk $(find $R/$O/t_xs$xs -name '*kernel_stats.csv') | cut -d, -f1-4)"
done
cd $R
for rep in 1 2 3; do
  for ext in head new; do
    if [ $ext = head ]; then export DGT_EXT_LIB=build/variants/head/_C.so; else unset DGT_EXT_LIB; fi
    timeout -k 10 200 python bench.py --model mlp --steps 200 --warmup 20 --no-sweep --no-secondary --no-baselines > $O/mlp_${ext}_$rep.json 2> $O/mlp_${ext}_$rep.err \
      || { tail -20 $O/mlp_${ext}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('mlp $ext', d['value'], d['ms_per_step'])" $O/mlp_${ext}_$rep.json
  done
done
unset DGT_EXT_LIB
DGT_GEMM_SK=1 timeout -k 10 200 python bench.py --model mlp --steps 200 --warmup 20 --no-sweep --no-secondary --no-baselines > $O/mlp_sk1.json 2> $O/mlp_sk1.err || { tail -20 $O/mlp_sk1.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('mlp new DGT_GEMM_SK=1 (NT forwards only)', d['value'], d['ms_per_step'])" $O/mlp_sk1.json
