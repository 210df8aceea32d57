# round 5: HIP graphs that captured a short chain of kernels launched as those kernels
# (_C.DirectLaunch) instead of replayed.  Arms: "fwd" = the default (one-kernel forward graphs of
# graph_module), "off" = DGT_GRAPH_DIRECT=0 (every graph replayed), "all8" = DGT_GRAPH_DIRECT_MAX=8
# (also the graphed tail and the whole-step graph).  Engine GPU tests first (default and all8), then
# interleaved fresh processes of the reference model's DeepSpeed-API loop, graph_module and the
# whole-step graph, then the per-call breakdown.
set -o pipefail
O=${OUT:-gpurun_out/r5dl}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_engine.py > $O/pytest_engine.log 2>&1 || { tail -40 $O/pytest_engine.log; exit 1; }
tail -1 $O/pytest_engine.log
DGT_GRAPH_DIRECT_MAX=8 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_engine.py > $O/pytest_engine_all8.log 2>&1 || { tail -40 $O/pytest_engine_all8.log; exit 1; }
tail -1 $O/pytest_engine_all8.log
for rep in 1 2 3 4; do
  for arm in fwd off all8; do
    case $arm in fwd) envs="" ;; off) envs="DGT_GRAPH_DIRECT=0" ;; all8) envs="DGT_GRAPH_DIRECT_MAX=8" ;; esac
    for cfg in configs/ds_graph_module.json configs/ds_graph_fused.json; do
      env $envs timeout -k 10 200 python bench.py --impl dgt-engine --deepspeed-config $cfg --steps 3000 --warmup 200 --no-sweep > $O/eng.json 2> $O/eng.err || { tail -20 $O/eng.err; exit 1; }
      python -c "import json; d=json.loads(open('$O/eng.json').read().splitlines()[-1]); print('$arm', '$cfg', d['value'], round(d['ms_per_step']*1e3,1), 'us/step', d['mean_loss'])" | tee -a $O/direct_ab.txt
    done
  done
done
for arm in fwd off all8; do
  case $arm in fwd) envs="" ;; off) envs="DGT_GRAPH_DIRECT=0" ;; all8) envs="DGT_GRAPH_DIRECT_MAX=8" ;; esac
  env $envs timeout -k 10 120 python scripts/engine_step_breakdown.py --steps 3000 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  grep "impl=" $O/b.log | sed "s/^/$arm /" | tee -a $O/direct_ab.txt
done
echo done
