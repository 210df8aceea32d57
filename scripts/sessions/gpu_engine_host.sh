#!/bin/bash
# Host-side cProfile of the generic engine's eager step per DeepSpeed config (scripts/engine_host_profile.py).
set -o pipefail
mkdir -p gpurun_out
for c in ds_zero0 ds_fused_linear ds_graph_module ds_zero1; do
  echo "== $c"
  timeout -k 10 180 python scripts/engine_host_profile.py --steps 3000 --config configs/$c.json --top 25 \
    > gpurun_out/engine_host_$c.txt 2>&1 || { tail -20 gpurun_out/engine_host_$c.txt; exit 1; }
  grep "engine-host" gpurun_out/engine_host_$c.txt
done
