#!/bin/bash
# Host wake-up after synchronize under HIP wait modes: probe, then bench.py at the driver's shape
# (K = 20, W = 5), interleaved fresh processes, REPS each.
set -o pipefail
mkdir -p gpurun_out
for mode in default spin envwait; do
  case $mode in
    default) E="" ;;
    spin) E="DGT_HIP_SPIN=1 DGT_HIP_WAIT=spin" ;;
    envwait) E="ROC_ACTIVE_WAIT_TIMEOUT=100000" ;;
  esac
  echo "== $mode"
  env $E timeout -k 10 120 python scripts/wait_mode_probe.py > gpurun_out/wm_$mode.log 2>&1 || { tail -5 gpurun_out/wm_$mode.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/wm_$mode.log
done
for r in $(seq ${REPS:-3}); do
  for mode in default spin envwait; do
    case $mode in
      default) E="" ;;
      spin) E="DGT_HIP_SPIN=1 DGT_HIP_WAIT=spin" ;;
      envwait) E="ROC_ACTIVE_WAIT_TIMEOUT=100000" ;;
    esac
    env $E timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/wm.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/wm.json').read().splitlines()[-1]); print('$mode', d['value'], round(d['ms_per_step'] * 1e3, 3), 'us/step')"
  done
done
