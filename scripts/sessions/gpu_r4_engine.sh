#!/bin/bash
# DeepSpeed-API engine on the reference SimpleNet (B = 4, fp32), per config, two interleaved reps,
# then a cProfile of the graph_module (graphed tail) step and a rocprofv3 kernel trace of it.
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for cfg in "" configs/ds_graph_module.json configs/ds_graph_fused.json; do
  timeout -k 10 200 python bench.py --impl dgt-engine ${cfg:+--deepspeed-config $cfg} --steps 3000 --warmup 200 --no-sweep > $O/eng.json 2> $O/eng.err || { tail -20 $O/eng.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/eng.json').read().splitlines()[-1]); print('${cfg:-eager}', d['value'], round(d['ms_per_step']*1e3,1), 'us/step', d['config']['impl'])" | tee -a $O/engine_paths.txt
done
done
timeout -k 10 200 python scripts/engine_host_profile.py --steps 3000 --config configs/ds_graph_module.json > $O/host_profile_graph_module.txt 2>&1 || { tail -20 $O/host_profile_graph_module.txt; exit 1; }
head -45 $O/host_profile_graph_module.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gm -o run -- python bench.py --impl dgt-engine --deepspeed-config configs/ds_graph_module.json --steps 2000 --warmup 100 --no-sweep > $O/prof_gm.log 2>&1 || { tail -20 $O/prof_gm.log; exit 1; }
f=$(find $O/prof_gm -name "*kernel_stats.csv" | head -1); cp "$f" $O/graph_module_kernel_stats.csv
cut -d, -f1-4 $O/graph_module_kernel_stats.csv | head -15
echo done
