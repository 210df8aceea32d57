# round 5: HIP runtime settings vs the device-side cost of a one-node graph replay (~10 us per replay
# against ~4.5 us for the same kernel launched directly, gpu_r5_launch_drain.sh): four probe
# processes per setting, interleaved.
set -o pipefail
O=${OUT:-gpurun_out/r5le}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4; do
  for arm in base flushexec0 capture0; do
    case $arm in
      base) envs="" ;;
      sysscope0) envs="ROC_SYSTEM_SCOPE_SIGNAL=0" ;;  # hangs the probe (host never sees the completion): not run
      flushexec0) envs="GPU_FLUSH_ON_EXECUTION=0" ;;
      capture0) envs="DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" ;;
    esac
    env $envs timeout -k 10 60 python scripts/graph_launch_probe.py > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
    grep launch-probe $O/p.log | sed "s/^/$arm /" | tee -a $O/env.txt
  done
done
echo done
