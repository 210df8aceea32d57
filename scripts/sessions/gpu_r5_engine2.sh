# round 5 (second half): the DeepSpeed-API engine on the reference SimpleNet after the host-path work
# (bound-input graphs, one-launch gather, pybind entry points, in-place gradients in captured
# backward, Adam advancing its own step counter): engine GPU tests, then REPS fresh processes per
# path, then the per-call breakdown of the graph_module loop.
set -o pipefail
O=${OUT:-gpurun_out/r5e3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_tiny_mlp.py > $O/pytest_engine.log 2>&1 || { tail -40 $O/pytest_engine.log; exit 1; }
tail -1 $O/pytest_engine.log
for rep in $(seq 1 ${REPS:-4}); do
for cfg in "" configs/ds_graph_module.json configs/ds_graph_fused.json; do
  timeout -k 10 200 python bench.py --impl dgt-engine ${cfg:+--deepspeed-config $cfg} --steps 3000 --warmup 200 --no-sweep > $O/eng.json 2> $O/eng.err || { tail -20 $O/eng.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/eng.json').read().splitlines()[-1]); print('${cfg:-eager}', d['value'], round(d['ms_per_step']*1e3,1), 'us/step', d['config']['impl'], d.get('engine_graph_replays'))" | tee -a $O/engine_paths.txt
done
done
for cfg in configs/ds_bench_mlp_fp32.json configs/ds_bench_mlp_bf16.json; do
  w=1024; [ "$cfg" = configs/ds_bench_mlp_bf16.json ] && w=4096
  timeout -k 10 200 python bench.py --model mlp --width $w --impl dgt-engine --deepspeed-config $cfg --steps 200 --warmup 20 --no-sweep > $O/mlp.json 2> $O/mlp.err || { tail -20 $O/mlp.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/mlp.json').read().splitlines()[-1]); print('$cfg', d['value'], round(d['ms_per_step']*1e3,1), 'us/step', d['model_tflops'], d['config']['impl'])" | tee -a $O/engine_paths.txt
done
for rep in 1 2; do
  timeout -k 10 120 python scripts/engine_step_breakdown.py --steps 3000 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  grep breakdown $O/b.log | tee -a $O/gm_breakdown.txt
done
timeout -k 10 200 python scripts/engine_host_profile.py --steps 3000 --config configs/ds_graph_module.json > $O/host_profile_graph_module.txt 2>&1 || { tail -20 $O/host_profile_graph_module.txt; exit 1; }
timeout -k 10 200 python scripts/engine_host_profile.py --steps 3000 > $O/host_profile_eager.txt 2>&1 || { tail -20 $O/host_profile_eager.txt; exit 1; }
echo done
