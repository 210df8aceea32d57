# round 5: is the slow launch mode host work or queue back-pressure?  Eight probe processes with the
# host cost of the first 32 launches after an idle sync, the steady host cost and the wall time per
# launch including the GPU's drain, for a direct kernel and a one-node graph replay.
set -o pipefail
O=${OUT:-gpurun_out/r5ld}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 60 python scripts/graph_launch_probe.py > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
  grep launch-probe $O/p.log | tee -a $O/drain.txt
done
echo done
