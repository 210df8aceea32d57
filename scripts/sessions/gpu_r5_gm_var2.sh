# round 5: per-call host time of the graph_module loop in several fresh processes (which call moves
# between a fast and a slow process), eager for comparison, then a kernel trace of the loop.
set -o pipefail
O=${OUT:-gpurun_out/r5v}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3 4 5 6; do
  timeout -k 10 120 python scripts/engine_step_breakdown.py --steps 3000 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  grep breakdown $O/b.log | tee -a $O/gm_breakdown.txt
done
for rep in 1 2; do
  timeout -k 10 120 python scripts/engine_step_breakdown.py --steps 3000 --config "" > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  grep breakdown $O/b.log | tee -a $O/gm_breakdown.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 scripts/engine_host_profile.py --steps 600 --config configs/ds_graph_module.json --no-cprofile > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep engine-host $O/trace.log
echo done
