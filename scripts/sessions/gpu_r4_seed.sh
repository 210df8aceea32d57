#!/bin/bash
# Unit-seed BCE backward: engine GPU tests, then the bf16 engine MLP bench x2 and its kernel trace.
set -o pipefail
O=gpurun_out/r4seed
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py tests/test_gemm_f32.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --model mlp --impl dgt-engine --steps 50 --warmup 10 --no-sweep > $O/eng.json 2> $O/eng.err || { tail -20 $O/eng.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/eng.json').read().strip().splitlines()[-1]); print('bf16 engine MLP', d['value'], d['ms_per_step'], d['config']['impl'])" | tee -a $O/eng.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --model mlp --impl dgt-engine --steps 20 --warmup 5 --no-sweep > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} $O/kernel_trace.csv
ls -la $O/kernel_trace.csv
