#!/bin/bash
# round 6: split-K 256x128 GEMM (variant 9) -- tests, per-product timing (both placements), the
# streaming probe, and the bf16 MLP step with the shape rule's split-K on / off.
set -o pipefail
O=gpurun_out/r6sk
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./build/bin/tile_stream > $O/tile_stream.jsonl 2>&1 || { tail -5 $O/tile_stream.jsonl; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gemm_sk.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python scripts/bench_gemm_sk.py > $O/gemm_xs1.jsonl 2>&1 || { tail -20 $O/gemm_xs1.jsonl; exit 1; }
DGT_GEMM_SK_XS=0 timeout -k 10 200 python scripts/bench_gemm_sk.py > $O/gemm_xs0.jsonl 2>&1 || { tail -20 $O/gemm_xs0.jsonl; exit 1; }
cat $O/gemm_xs1.jsonl $O/gemm_xs0.jsonl
for rep in 1 2; do
  for sk in 0 1; do
    DGT_GEMM_SK=$sk timeout -k 10 200 python bench.py --model mlp --steps 200 --warmup 20 --no-sweep --no-secondary --no-baselines > $O/mlp_sk${sk}_$rep.json 2> $O/mlp_sk${sk}_$rep.err \
      || { tail -20 $O/mlp_sk${sk}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('mlp sk=$sk', d['value'], d['ms_per_step'])" $O/mlp_sk${sk}_$rep.json
  done
done
