#!/bin/bash
# round 6: split-K v2 (per-row-half meeting, sc1 hand-off, no fences) + epilogue bias prefetch in
# every staged-epilogue kernel: tests, per-product timing, loop / half-epilogue diagnostics, MLP step.
set -o pipefail
O=gpurun_out/${SKO:-r6sk3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gemm_sk.py tests/test_mlp_gemm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python scripts/bench_gemm_sk.py > $O/gemm_xs1.jsonl 2>&1 || { tail -20 $O/gemm_xs1.jsonl; exit 1; }
DGT_GEMM_SK_XS=0 timeout -k 10 200 python scripts/bench_gemm_sk.py > $O/gemm_xs0.jsonl 2>&1 || { tail -20 $O/gemm_xs0.jsonl; exit 1; }
cat $O/gemm_xs1.jsonl $O/gemm_xs0.jsonl | grep -v amdgpu.ids
R=$GRAFT_REPO_ROOT
cd /tmp
for xs in 1 3 5; do
  DGT_GEMM_SK_XS=$xs timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/t_xs$xs -o run -- \
    python3 $R/scripts/gemm_one.py 1024 4096 4096 9 30 fwd > $R/$O/t_xs$xs.log 2>&1 || { echo "xs $xs failed"; tail -5 $R/$O/t_xs$xs.log; exit 1; }
  echo "xs=$xs $(grep -h gemm_nt_sk $(find $R/$O/t_xs$xs -name '*kernel_stats.csv') | cut -d, -f1-4)"
done
cd $R
for rep in 1 2; do
  for sk in 0 1; do
    DGT_GEMM_SK=$sk timeout -k 10 200 python bench.py --model mlp --steps 200 --warmup 20 --no-sweep --no-secondary --no-baselines > $O/mlp_sk${sk}_$rep.json 2> $O/mlp_sk${sk}_$rep.err \
      || { tail -20 $O/mlp_sk${sk}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('mlp sk=$sk', d['value'], d['ms_per_step'])" $O/mlp_sk${sk}_$rep.json
  done
done
