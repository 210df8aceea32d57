# round 5: graph_module with bound inputs (graphs that read a recurring input address in place),
# the one-launch batch gather (data.gather_batch) and the C++ Function.apply entry: the engine GPU
# tests, then the per-call breakdown and the engine bench paths in fresh processes.
set -o pipefail
O=${OUT:-gpurun_out/r5b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine.py > $O/pytest_engine.log 2>&1 || { tail -40 $O/pytest_engine.log; exit 1; }
tail -1 $O/pytest_engine.log
for rep in 1 2 3 4; do
  timeout -k 10 120 python scripts/engine_step_breakdown.py --steps 3000 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  grep breakdown $O/b.log | tee -a $O/gm_breakdown.txt
done
for rep in 1 2 3 4; do
for cfg in "" configs/ds_graph_module.json; do
  timeout -k 10 200 python bench.py --impl dgt-engine ${cfg:+--deepspeed-config $cfg} --steps 3000 --warmup 200 --no-sweep > $O/eng.json 2> $O/eng.err || { tail -20 $O/eng.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/eng.json').read().splitlines()[-1]); print('${cfg:-eager}', d['value'], round(d['ms_per_step']*1e3,1), 'us/step', d['config']['impl'], d.get('engine_graph_replays'))" | tee -a $O/engine_paths.txt
done
done
echo done
