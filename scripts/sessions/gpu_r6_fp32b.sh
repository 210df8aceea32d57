#!/bin/bash
# round 6: the fp32 engine MLP (SyntheticMLP(1024, 4) on the exact-fp32 GEMM) at per-GPU batch 256 / 1024
# against torch fp32 -- does a small batch leave the fp32 GEMM's grid under-filled?
set -o pipefail
O=gpurun_out/r6fp32b; mkdir -p gpurun_out/r6fp32p
mkdir -p $O
export TMPDIR=/tmp
for B in ${BATCHES:-256 1024}; do
  timeout -k 10 200 python bench.py --model mlp --impl dgt-engine --width 1024 --batch $B --deepspeed-config configs/ds_bench_mlp_fp32.json \
    --steps 200 --warmup 20 --no-sweep --no-secondary --no-baselines > $O/ours_$B.json 2> $O/ours_$B.err || { tail -20 $O/ours_$B.err; exit 1; }
  timeout -k 10 200 python bench.py --model mlp --impl engine --torch-dtype fp32 --width 1024 --batch $B \
    --steps 100 --warmup 20 --no-sweep --no-secondary --no-baselines > $O/torch_$B.json 2> $O/torch_$B.err || { tail -20 $O/torch_$B.err; exit 1; }
  python -c "import json,sys; f=lambda p: json.loads([l for l in open(p) if l.startswith('{')][-1]); a=f(sys.argv[1]); b=f(sys.argv[2]); print('B', $B, 'ours', a['value'], a['ms_per_step'], 'torch', b['value'], b['ms_per_step'])" $O/ours_$B.json $O/torch_$B.json
done
# kernel stats at B = 256 (the head's kernel choice shows here)
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6fp32p/p -o run -- python bench.py --model mlp --impl dgt-engine --width 1024 --batch 256 \
  --deepspeed-config configs/ds_bench_mlp_fp32.json --steps 100 --warmup 10 --no-sweep --no-secondary --no-baselines > gpurun_out/r6fp32p/out.log 2>&1
