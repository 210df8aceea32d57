#!/bin/bash
# round 6: the bf16 MLP (SyntheticMLP(4096, 4)) at per-GPU batch 256 / 512 -- MLPTrainer and the
# DeepSpeed-style engine with the small-grid split-K mode on / off, and torch bf16 autocast.
set -o pipefail
O=gpurun_out/r6smallb
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, env..., args...
  local name=$1; shift
  timeout -k 10 200 env "$@" > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/$name.json $name
}
for B in 256 512; do
  for skn in 1 0; do
    run mlp_b${B}_skn$skn DGT_GEMM_SKN=$skn python bench.py --model mlp --batch $B --steps 200 --warmup 20 --no-sweep --no-secondary --no-baselines
    run engine_b${B}_skn$skn DGT_GEMM_SKN=$skn python bench.py --model mlp --impl dgt-engine --batch $B --steps 200 --warmup 20 --no-sweep --no-secondary --no-baselines
  done
  run torch_b${B} DGT_GEMM_SKN=1 python bench.py --model mlp --impl engine --batch $B --steps 100 --warmup 20 --no-sweep --no-secondary --no-baselines
done
