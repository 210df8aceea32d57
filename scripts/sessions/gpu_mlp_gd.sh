#!/bin/bash
# MLP: bf16 vs fp32 weight gradients (tests + interleaved bench + profile of the default).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_mlp_gemm.py tests/test_gpu_multiproc.py -x -q -m gpu -k "not eight_ranks and not many_ranks" --timeout 300 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_mlp.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for gd in fp32 bf16; do
    DGT_MLP_GRAD_DTYPE=$gd timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 > gpurun_out/gd.json 2> gpurun_out/gd.err || { tail -20 gpurun_out/gd.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/gd.json')); print('$gd', d['value'], d['ms_per_step'], d['model_tflops'], d['mean_loss'])" | tee -a gpurun_out/mlp_gd.txt
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mlp -o run -- python bench.py --model mlp --steps 20 --warmup 5 > gpurun_out/prof_mlp.log 2>&1 || { tail -20 gpurun_out/prof_mlp.log; exit 1; }
