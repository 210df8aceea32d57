#!/bin/bash
# The DeepSpeed-API eager loop on the reference model: cProfile of the host side and its kernel list.
set -o pipefail
O=gpurun_out/r4ep
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python scripts/engine_host_profile.py --steps 3000 > $O/host_profile_eager.txt 2>&1 || { tail -20 $O/host_profile_eager.txt; exit 1; }
head -50 $O/host_profile_eager.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --impl dgt-engine --steps 2000 --warmup 100 --no-sweep > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/eager_kernel_stats.csv
cut -d, -f1-4 $O/eager_kernel_stats.csv | head -15
