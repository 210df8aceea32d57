#!/bin/bash
# Engine deferred gradient-bucket zeroing: engine GPU tests, then the DeepSpeed-API MLP bench and
# its kernel stats.  Outputs gpurun_out/dz/.
set -o pipefail
mkdir -p gpurun_out/dz
export TMPDIR=/tmp
O=gpurun_out/dz
timeout -k 10 600 python -u -m pytest -v tests/test_gpu_engine.py tests/test_gpu_train.py -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $O/pytest.log | head; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model mlp --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_bf16.json --steps 50 --warmup 10 > $O/bench_engine_$i.json 2> $O/bench_engine_$i.err || { tail -20 $O/bench_engine_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_engine_$i.json')); print(d['value'], d['ms_per_step'], d.get('model_tflops'))"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --model mlp --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_bf16.json --steps 20 --warmup 5 --no-sweep > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo done
