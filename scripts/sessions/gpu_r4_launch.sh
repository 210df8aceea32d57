#!/bin/bash
# Prepared fused launch: bitwise test, launch probe, 8 driver-shape fresh processes.
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiny_mlp.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 200 python scripts/headline_launch_probe.py > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.jsonl
: > $O/driver8.txt
for i in 1 2 3 4 5 6 7 8; do
  DGT_BENCH_BREAKDOWN=1 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.json 2> $O/drv_$i.err || { tail -20 $O/drv_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/drv_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" | tee -a $O/driver8.txt
  grep "timed region" $O/drv_$i.err | tee -a $O/driver8.txt
done
python - <<'PY'
import statistics
v=[float(l.split()[0]) for l in open('gpurun_out/r4l/driver8.txt') if l[0].isdigit()]
print('median', statistics.median(v), 'min', min(v), 'max', max(v))
PY
timeout -k 10 300 python bench.py --steps 20000 --warmup 100 > $O/longk.json 2> $O/longk.err || { tail -20 $O/longk.err; exit 1; }
python -c "import json; d=json.loads(open('$O/longk.json').read().strip().splitlines()[-1]); print('long K', d['value'], d['ms_per_step'], d['mean_loss'])"
