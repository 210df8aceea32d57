#!/bin/bash
# bf16 MLP step: the fused wgrad+Adam in line (default) vs on a side stream beside the dgrads, with
# 128 KiB-LDS kernels (one block per CU) or 64 KiB ones (variant 1: two kernels' blocks share a CU).
# Interleaved fresh-process runs; bench.py --model mlp, 50 steps.
set -o pipefail
mkdir -p gpurun_out/side
export TMPDIR=/tmp
run() {  # run <tag> <env...>
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --model mlp --steps 50 --warmup 10 --no-sweep > gpurun_out/side/$tag.json 2> gpurun_out/side/$tag.err || { tail -5 gpurun_out/side/$tag.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/side/$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
}
timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_mlp_gemm.py -k "trainer or fused" > gpurun_out/side/pytest.log 2>&1 || { tail -20 gpurun_out/side/pytest.log; exit 1; }
tail -1 gpurun_out/side/pytest.log
for r in 1 2; do
  run inline_$r DGT_MLP_WGA_SIDE=0 || exit 1
  run side_v0_$r DGT_MLP_WGA_SIDE=1 || exit 1
  run side_v1v1_$r DGT_MLP_WGA_SIDE=1 DGT_MLP_WGA_VARIANT=1 DGT_MLP_DGRAD_VARIANT=1 || exit 1
  run side_wga1_$r DGT_MLP_WGA_SIDE=1 DGT_MLP_WGA_VARIANT=1 || exit 1
  run inline_wga1_$r DGT_MLP_WGA_SIDE=0 DGT_MLP_WGA_VARIANT=1 || exit 1
done
