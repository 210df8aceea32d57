#!/bin/bash
# bf16 MLP through the DeepSpeed-style engine vs the trainer: benches + the engine's kernel trace.
set -o pipefail
O=gpurun_out/r4be2
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py --model mlp --impl dgt-engine --steps 50 --warmup 10 --no-sweep > $O/eng.json 2> $O/eng.err || { tail -20 $O/eng.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/eng.json').read().strip().splitlines()[-1]); print('bf16 engine MLP', d['value'], d['ms_per_step'], d['config']['impl'])"
  timeout -k 10 300 python bench.py --model mlp --steps 50 --warmup 10 --no-sweep > $O/tr.json 2> $O/tr.err || { tail -20 $O/tr.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/tr.json').read().strip().splitlines()[-1]); print('bf16 trainer MLP', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --model mlp --impl dgt-engine --steps 20 --warmup 5 --no-sweep > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} $O/kernel_trace.csv
ls -la $O/kernel_trace.csv
