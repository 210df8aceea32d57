#!/bin/bash
# Full GPU session: test suite, smoke, headline bench, MLP bench, exchange rehearsals, rocprof stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "== bench default"
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print(d['value'], d['ms_per_step'])"
echo "== bench, the driver's shape"
for i in 1 2 3; do
  DGT_BENCH_BREAKDOWN=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver_$i.json 2> gpurun_out/bench_driver_$i.err || { tail -20 gpurun_out/bench_driver_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_driver_$i.json')); print(d['value'], d['ms_per_step'])"
done
echo "== bench mlp"
timeout -k 10 300 python bench.py --model mlp --steps 100 --warmup 10 > gpurun_out/bench_mlp.json 2> gpurun_out/bench_mlp.err || { tail -20 gpurun_out/bench_mlp.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_mlp.json')); print(d['value'], d['ms_per_step'], d['model_tflops'])"
echo "== exchange rehearsals"
bash scripts/gpu_xch_bench.sh || exit 1
echo "== rocprof fused"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fused -o run -- python bench.py --steps 100000 --warmup 5000 > gpurun_out/prof_fused.log 2>&1 || { tail -20 gpurun_out/prof_fused.log; exit 1; }
echo "== rocprof mlp"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mlp -o run -- python bench.py --model mlp --steps 20 --warmup 5 > gpurun_out/prof_mlp.log 2>&1 || { tail -20 gpurun_out/prof_mlp.log; exit 1; }
echo done
