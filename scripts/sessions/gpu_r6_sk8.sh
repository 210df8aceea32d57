#!/bin/bash
# round 6: per-kernel durations inside the bf16 MLP step with the shape rule's split-K on / off
set -o pipefail
O=gpurun_out/r6sk8
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for sk in 0 1; do
  DGT_GEMM_SK=$sk timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/sk$sk -o run -- \
    python3 $R/bench.py --model mlp --steps 200 --warmup 20 --no-sweep --no-secondary --no-baselines > $R/$O/sk$sk.log 2>&1 || { echo "sk $sk failed"; tail -5 $R/$O/sk$sk.log; exit 1; }
  echo "sk=$sk"; grep -h "gemm_nt" $(find $R/$O/sk$sk -name '*kernel_stats.csv') | cut -d, -f1-4,6,7
done
