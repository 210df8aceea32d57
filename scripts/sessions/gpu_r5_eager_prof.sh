# round 5: host profile (cProfile) of the eager DeepSpeed-API step and the graph_module step on the
# reference model (scripts/engine_host_profile.py)
set -o pipefail
O=gpurun_out/r5ep
mkdir -p $O
timeout -k 10 200 python scripts/engine_host_profile.py --steps 3000 --top 45 > $O/eager.txt 2>&1 || { tail -20 $O/eager.txt; exit 1; }
timeout -k 10 200 python scripts/engine_host_profile.py --steps 3000 --top 45 --config configs/ds_graph_module.json > $O/gm.txt 2>&1 || { tail -20 $O/gm.txt; exit 1; }
grep "engine-host" $O/eager.txt $O/gm.txt
