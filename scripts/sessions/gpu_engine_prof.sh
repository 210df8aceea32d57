#!/bin/bash
# Engine path (DeepSpeed-style initialize() on the nn.Module): bench + kernel stats, eager and HIP-graph.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in ${@:-configs/ds_zero0.json configs/ds_graph.json configs/ds_graph_fused.json}; do
  n=$(basename $cfg .json)
  timeout -k 10 200 python bench.py --impl dgt-engine --deepspeed-config $cfg --steps 3000 --warmup 300 > gpurun_out/eng_$n.json 2> gpurun_out/eng_$n.err || { tail -20 gpurun_out/eng_$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/eng_$n.json')); print('$n', d['value'], d['ms_per_step'], d['config']['impl'])"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_eng_$n -o run -- python bench.py --impl dgt-engine --deepspeed-config $cfg --steps 1000 --warmup 100 > gpurun_out/prof_eng_$n.log 2>&1 || { tail -20 gpurun_out/prof_eng_$n.log; exit 1; }
done
