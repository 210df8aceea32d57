# round 5: HIP runtime settings vs the per-node cost of graph-launched kernels (every node of the
# engine's graphs takes ~4.5 us under the profiler, the same kernels ~2.8 us launched eagerly):
# whole-step graph and graph_module bench per setting, 2 fresh processes each.
set -o pipefail
O=${OUT:-gpurun_out/r5e2}
mkdir -p $O
export TMPDIR=/tmp
run() {  # label, env...
  local label=$1; shift
  for rep in 1 2; do
    for cfg in configs/ds_graph_fused.json configs/ds_graph_module.json; do
      env "$@" timeout -k 10 120 python bench.py --impl dgt-engine --deepspeed-config $cfg --steps 3000 --warmup 200 --no-sweep > $O/eng.json 2> $O/eng.err || { tail -20 $O/eng.err; exit 1; }
      python -c "import json; d=json.loads(open('$O/eng.json').read().splitlines()[-1]); print('$label', '$cfg', d['value'], round(d['ms_per_step']*1e3,1), 'us/step')" | tee -a $O/graph_env.txt
    done
  done
}
run base DGT_NOP=1
run packet_capture_0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run packet_capture_1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run dev_kernarg_1 HIP_FORCE_DEV_KERNARG=1
run dev_kernarg_0 HIP_FORCE_DEV_KERNARG=0
run graph_batch_1 DEBUG_HIP_GRAPH_BATCH_SIZE=1
run graph_batch_64 DEBUG_HIP_GRAPH_BATCH_SIZE=64
echo done
