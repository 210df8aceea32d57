#!/bin/bash
# round 6, session H: new engine tests (retained fused BCE under graph_module, concurrent stream probe),
# the fuzz file's durations, MLP trainer overlap schedule with forced collectives.
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine_fuzz.py tests/test_gpu_engine.py tests/test_gpu_force_collectives.py \
  -m gpu -v --durations=20 --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -28 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
for s in overlap flat; do
  DGT_FORCE_COLLECTIVES=1 timeout -k 10 120 python bench.py --model mlp --schedule $s --steps 100 --warmup 20 --no-sweep \
    2>/dev/null | grep "^{" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$s', d['value'], d['ms_per_step'], d['config']['exchange'])" || exit 1
done
