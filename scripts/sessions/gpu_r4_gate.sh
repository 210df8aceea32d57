#!/bin/bash
# Round-4 gate on one MI355X, in the driver's own form: the whole GPU suite in ONE pytest process
# (no --ignore, -x, alphabetical order as the driver runs it), smoke(), the driver's bench command,
# then a self-launched multi-rank rehearsal on the one card (bench.py --gpus 4 with no torchrun:
# bench.py starts its own ranks).  Outputs under gpurun_out/r4g/.
set -o pipefail
O=gpurun_out/r4g
mkdir -p $O
export TMPDIR=/tmp
echo "== pytest -m gpu (one process, the driver's form)"
timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; exit $rc; }
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "== bench, the driver's command"
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || { tail -20 $O/bench_driver_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_driver_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
done
echo "== self-launched 4-rank rehearsal on one card"
DGT_ALLOW_OVERSUBSCRIBE=1 timeout -k 10 400 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/bench_self4.json 2> $O/bench_self4.err || { tail -30 $O/bench_self4.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_self4.json').read().strip().splitlines()[-1]); print(d['value'], d['ranks'], d['config']['parallelism'], len(d['oneshot_xgmi_sweep']), d['allreduce_busbw_GBps'])"
echo done
