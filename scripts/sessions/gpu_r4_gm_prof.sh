#!/bin/bash
# Host profile of the graph_module engine loop on the reference model (twice: the run-to-run spread).
set -o pipefail
O=gpurun_out/r4gm
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python scripts/engine_host_profile.py --steps 3000 --config configs/ds_graph_module.json --top 25 > $O/host_gm_$i.txt 2>&1 || { tail -20 $O/host_gm_$i.txt; exit 1; }
  grep -v amdgpu.ids $O/host_gm_$i.txt | head -40
done
