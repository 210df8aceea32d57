#!/bin/bash
# Kernel stats of the bench-size MLP for the tree in _ab/ and this tree (rocprofv3 --kernel-trace --stats).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in _ab .; do
  n=$([ "$t" = "." ] && echo new || echo ab)
  (cd $t && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_mlp_$n -o run -- python bench.py --model mlp --steps 40 --warmup 5 --no-sweep > $GRAFT_REPO_ROOT/gpurun_out/prof_mlp_$n.log 2>&1) || { tail -20 gpurun_out/prof_mlp_$n.log; exit 1; }
done
