# round 5: kernel trace of the graph_module engine loop (per-step kernels and gaps) and of the
# whole-step graph, after the bound-input / in-place-gradient changes
set -o pipefail
O=${OUT:-gpurun_out/r5t}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_tiny_mlp.py > $O/pytest_engine.log 2>&1 || { tail -40 $O/pytest_engine.log; exit 1; }
tail -1 $O/pytest_engine.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/gm -o run -- python3 scripts/engine_host_profile.py --steps 600 --config configs/ds_graph_module.json --no-cprofile > $O/gm.log 2>&1 || { tail -20 $O/gm.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/whole -o run -- python3 scripts/engine_host_profile.py --steps 600 --config configs/ds_graph_fused.json --no-cprofile > $O/whole.log 2>&1 || { tail -20 $O/whole.log; exit 1; }
grep engine-host $O/gm.log $O/whole.log
for rep in 1 2 3; do
for cfg in configs/ds_graph_module.json configs/ds_graph_fused.json; do
  timeout -k 10 200 python bench.py --impl dgt-engine --deepspeed-config $cfg --steps 3000 --warmup 200 --no-sweep > $O/eng.json 2> $O/eng.err || { tail -20 $O/eng.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/eng.json').read().splitlines()[-1]); print('$cfg', d['value'], round(d['ms_per_step']*1e3,1), 'us/step', d['config']['impl'], d.get('engine_graph_replays'))" | tee -a $O/engine_paths.txt
done
done
echo done
