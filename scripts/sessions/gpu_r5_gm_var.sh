# round 5: why the graph_module engine path varies 49-82 us/step between processes on one box.
# Per HIP runtime setting, fresh processes of scripts/engine_host_profile.py (host enqueue time vs
# total), then a kernel trace of the graph_module loop (per-step device span and gaps).
set -o pipefail
O=${OUT:-gpurun_out/r5v}
mkdir -p $O
export TMPDIR=/tmp
run() {  # label, env...
  local label=$1; shift
  for rep in 1 2 3; do
    env "$@" timeout -k 10 120 python scripts/engine_host_profile.py --steps 3000 --config configs/ds_graph_module.json --no-cprofile > $O/v.log 2>&1 || { tail -20 $O/v.log; exit 1; }
    echo "$label $(grep engine-host $O/v.log)" | tee -a $O/gm_var.txt
  done
}
run base DGT_NOP=1
run packet_capture_0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run packet_capture_1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run force_graph_queues_0 DEBUG_HIP_FORCE_GRAPH_QUEUES=0
run force_graph_queues_1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1
run dev_kernarg_1 HIP_FORCE_DEV_KERNARG=1
for rep in 1 2; do
  timeout -k 10 120 python scripts/engine_host_profile.py --steps 3000 --config configs/ds_graph_fused.json --no-cprofile > $O/v.log 2>&1 || { tail -20 $O/v.log; exit 1; }
  echo "whole_step_graph $(grep engine-host $O/v.log)" | tee -a $O/gm_var.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 scripts/engine_host_profile.py --steps 600 --config configs/ds_graph_module.json --no-cprofile > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep engine-host $O/trace.log
echo done
