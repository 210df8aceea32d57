# round 5: where is the graph_module loop's process-to-process spread?  Six fresh processes of the
# launch probe (direct kernel vs one-node graph replay, default vs created stream), then the per-call
# breakdown on the default stream and on a created stream, alternating, four processes each.
set -o pipefail
O=${OUT:-gpurun_out/r5lv}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4 5 6; do
  timeout -k 10 120 python scripts/graph_launch_probe.py > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
  grep launch-probe $O/p.log | tee -a $O/launch_var.txt
done
for i in 1 2 3 4; do
  for arm in "" --side-stream; do
    timeout -k 10 120 python scripts/engine_step_breakdown.py --steps 3000 $arm > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    grep "impl=" $O/b.log | tee -a $O/launch_var.txt
  done
done
echo done
