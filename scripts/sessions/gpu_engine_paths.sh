#!/bin/bash
# The generic engine (initialize() on the reference nn.Module) per DeepSpeed config, REPS
# interleaved runs: eager, eager + fused_linear, graph_module (eager API, graphed module), whole-
# step HIP graph, whole-step graph + fused_linear.  Then a rocprofv3 kernel trace of the eager path.
set -o pipefail
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
for cfg in "" configs/ds_fused_linear.json configs/ds_graph_module.json configs/ds_graph.json configs/ds_graph_fused.json; do
  timeout -k 10 200 python bench.py --impl dgt-engine ${cfg:+--deepspeed-config $cfg} --steps 3000 --warmup 200 --no-sweep > gpurun_out/eng.json 2> gpurun_out/eng.err || { tail -20 gpurun_out/eng.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/eng.json').read().splitlines()[-1]); print('${cfg:-eager}', d['value'], round(d['ms_per_step']*1e3,1), 'us/step')"
done
done
if [ -n "$PROF" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_eng -o run -- python bench.py --impl dgt-engine ${PROF_CFG:+--deepspeed-config $PROF_CFG} --steps 2000 --warmup 100 --no-sweep > gpurun_out/prof_eng.log 2>&1
fi
