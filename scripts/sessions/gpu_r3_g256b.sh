#!/bin/bash
# The asm-DMA 256x256 kernel as the only form: GEMM + engine tests, the 256 kernel vs hipBLASLt,
# and the MLP step (trainer and DeepSpeed-API engine).
set -o pipefail
mkdir -p gpurun_out/g256b
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_mlp_gemm.py tests/test_gpu_engine.py > gpurun_out/g256b/pytest.log 2>&1 || { tail -30 gpurun_out/g256b/pytest.log; exit 1; }
tail -1 gpurun_out/g256b/pytest.log
timeout -k 10 300 python scripts/bench_gemm256_ab.py > gpurun_out/g256b/ab.jsonl 2> gpurun_out/g256b/ab.err || { tail -20 gpurun_out/g256b/ab.err; exit 1; }
cat gpurun_out/g256b/ab.jsonl
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model mlp --steps 50 --warmup 10 --no-sweep > gpurun_out/g256b/mlp_$i.json 2> gpurun_out/g256b/mlp_$i.err || { tail -20 gpurun_out/g256b/mlp_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/g256b/mlp_$i.json')); print('mlp run $i', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --model mlp --impl dgt-engine --steps 30 --warmup 10 --no-sweep > gpurun_out/g256b/eng.json 2> gpurun_out/g256b/eng.err || { tail -20 gpurun_out/g256b/eng.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/g256b/eng.json')); print('engine mlp', d['value'], d['ms_per_step'])"
