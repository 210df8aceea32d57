#!/bin/bash
# fp32 deferred zeroing + direct backward: engine GPU tests, the eager engine on the reference model,
# the graph_module engine, and the fp32 engine MLP.
set -o pipefail
O=gpurun_out/r4d32
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py tests/test_gemm_f32.py tests/test_gpu_train.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --impl dgt-engine --steps 3000 --warmup 200 --no-sweep > $O/eager.json 2> $O/eager.err || { tail -20 $O/eager.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/eager.json').read().strip().splitlines()[-1]); print('eager', d['value'], d['ms_per_step']*1e3, 'us/step', d['config']['impl'])" | tee -a $O/engine.txt
  timeout -k 10 200 python bench.py --impl dgt-engine --deepspeed-config configs/ds_graph_module.json --steps 3000 --warmup 200 --no-sweep > $O/gm.json 2> $O/gm.err || { tail -20 $O/gm.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/gm.json').read().strip().splitlines()[-1]); print('graph_module', d['value'], d['ms_per_step']*1e3, 'us/step', d['config']['impl'])" | tee -a $O/engine.txt
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --model mlp --width 1024 --depth 4 --batch 1024 --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 50 --warmup 10 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/mlp.json').read().strip().splitlines()[-1]); print('fp32 engine MLP', d['value'], d['ms_per_step'])" | tee -a $O/engine.txt
done
