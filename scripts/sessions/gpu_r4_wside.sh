#!/bin/bash
# wgrad beside dgrad on a side stream (DGT_MLP_WGRAD_SIDE): bitwise test, interleaved MLP A/B, and
# the launch probe with the bench's own launch sequence.
set -o pipefail
O=gpurun_out/r4w
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mlp_gemm.py -x -q --timeout 120 --timeout-method thread -k "side_stream" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; exit $rc; }
: > $O/mlp_ab.txt
for rep in 1 2 3; do
for v in 0 1; do
  DGT_MLP_WGRAD_SIDE=$v timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print('wgrad_side $v', d['value'], d['ms_per_step'], d['model_tflops'])" | tee -a $O/mlp_ab.txt
done
done
timeout -k 10 200 python scripts/headline_launch_probe.py > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.jsonl
