#!/bin/bash
# Round-5 gate on one MI355X in the driver's own form: the whole GPU suite in ONE pytest process,
# smoke(), the driver's bench command three times (headline + the bf16 / fp32 MLP blocks), a rocprofv3
# kernel-stats run of the driver's bench command, then a self-launched 4-rank rehearsal on the one card.
set -o pipefail
O=${OUT:-gpurun_out/r5g}
mkdir -p $O
export TMPDIR=/tmp
echo "== pytest -m gpu (one process, the driver's form)"
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; exit $rc; }
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "== bench, the driver's command"
for i in 1 2 3; do
  t0=$(date +%s.%N)
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || { tail -20 $O/bench_driver_$i.err; exit 1; }
  echo "wall $(python -c "print(round($(date +%s.%N) - $t0, 1))") s"
  python -c "import json; d=json.loads(open('$O/bench_driver_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k: (d[k].get('iters_per_s'), d[k].get('model_tflops'), d[k].get('block_wall_s'), d[k].get('error')) for k in ('bf16_mlp', 'fp32_engine_mlp')})"
done
echo "== rocprofv3 kernel stats of the driver's command"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_driver.log 2>&1 || { tail -20 $O/prof_driver.log; exit 1; }
echo "== self-launched 4-rank rehearsal on one card"
DGT_ALLOW_OVERSUBSCRIBE=1 timeout -k 10 400 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/bench_self4.json 2> $O/bench_self4.err || { tail -30 $O/bench_self4.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_self4.json').read().strip().splitlines()[-1]); print(d['value'], d['ranks'], d['config']['parallelism'], len(d['oneshot_xgmi_sweep']), d['allreduce_busbw_GBps'], d['hung'])"
echo done
