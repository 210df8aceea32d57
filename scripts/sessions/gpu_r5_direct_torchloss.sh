# round 5: graph_module with the reference's own criterion (torch.nn.BCEWithLogitsLoss: autograd
# backward through the graphed backward, eager fused Adam, no graphed tail), graphs launched as their
# kernels (default) vs replayed (DGT_GRAPH_DIRECT=0), interleaved fresh processes.
set -o pipefail
O=${OUT:-gpurun_out/r5dt}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3 4; do
  for arm in 1 0; do
    DGT_GRAPH_DIRECT=$arm timeout -k 10 120 python scripts/engine_step_breakdown.py --steps 3000 --torch-loss > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    grep "impl=" $O/b.log | sed "s/^/direct=$arm /" | tee -a $O/torchloss_ab.txt
  done
done
echo done
