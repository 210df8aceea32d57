#!/bin/bash
# Round-3 validation session on one MI355X: every single-GPU test, smoke, the headline bench at
# default and driver shapes, the bf16 MLP (MLPTrainer and the DeepSpeed-API engine), and rocprofv3
# kernel stats of both MLP paths (the engine trace must hold no hipBLASLt Cijk_* kernel).
# Outputs under gpurun_out/r3f/.  (Multi-rank rehearsals: scripts/gpu_r3_xch.sh.)
set -o pipefail
mkdir -p gpurun_out/r3f
export TMPDIR=/tmp
O=gpurun_out/r3f
echo "== pytest gpu (single GPU)"
timeout -k 10 900 python -u -m pytest tests -q -m gpu --ignore tests/test_gpu_multiproc.py --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; exit $rc; }
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "== bench default"
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['ms_per_step'])"
echo "== bench, the driver's shape"
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || { tail -20 $O/bench_driver_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$i.json')); print(d['value'], d['ms_per_step'])"
done
echo "== bench mlp (MLPTrainer)"
for i in 1 2; do
  timeout -k 10 300 python bench.py --model mlp --steps 100 --warmup 10 > $O/bench_mlp_$i.json 2> $O/bench_mlp_$i.err || { tail -20 $O/bench_mlp_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_mlp_$i.json')); print(d['value'], d['ms_per_step'], d.get('model_tflops'))"
done
echo "== bench mlp (DeepSpeed-API engine, bf16 MFMA chain)"
timeout -k 10 300 python bench.py --model mlp --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_bf16.json --steps 50 --warmup 10 > $O/bench_mlp_engine.json 2> $O/bench_mlp_engine.err || { tail -20 $O/bench_mlp_engine.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_mlp_engine.json')); print(d['value'], d['ms_per_step'], d.get('model_tflops'))"
echo "== rocprof mlp engine"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp_engine -o run -- python bench.py --model mlp --impl dgt-engine --deepspeed-config configs/ds_bench_mlp_bf16.json --steps 20 --warmup 5 --no-sweep > $O/prof_mlp_engine.log 2>&1 || { tail -20 $O/prof_mlp_engine.log; exit 1; }
echo "== rocprof mlp trainer"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o run -- python bench.py --model mlp --steps 20 --warmup 5 --no-sweep > $O/prof_mlp.log 2>&1 || { tail -20 $O/prof_mlp.log; exit 1; }
echo done
