# round 5: HIP runtime settings vs the headline's fixed launch -> completion cost at the driver's
# shape (bench.py --gpus 1 --steps 20 --warmup 5: one launch + one synchronisation), interleaved
# fresh processes: defaults, kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1 / =0),
# one hardware queue (GPU_MAX_HW_QUEUES=1).  --no-secondary: the headline line only.
set -o pipefail
O=${OUT:-gpurun_out/r5h}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3 4; do
  for arm in base kernarg1 kernarg0 hwq1; do
    case $arm in base) e="DGT_NOP=1";; kernarg1) e="HIP_FORCE_DEV_KERNARG=1";; kernarg0) e="HIP_FORCE_DEV_KERNARG=0";; hwq1) e="GPU_MAX_HW_QUEUES=1";; esac
    env $e timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary > $O/h.json 2> $O/h.err || { tail -20 $O/h.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/h.json').read().splitlines()[-1]); print('$arm', d['value'], round(d['ms_per_step']*1e3, 3), 'us/step')" | tee -a $O/headline_env.txt
  done
done
echo done
