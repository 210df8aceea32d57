#!/bin/bash
# Round-4 perf pass 1: fp32 MFMA GEMM numbers + engine paths (graphed tail) + the L2->LDS streaming
# microbenchmark.  Each step under its own time limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out/r4s
bash scripts/gpu_r4_f32.sh || exit 1
bash scripts/gpu_r4_engine.sh || exit 1
echo "== panel_stream"
timeout -k 10 120 ./build/bin/panel_stream > gpurun_out/r4s/panel_stream.jsonl 2>&1 || { tail -20 gpurun_out/r4s/panel_stream.jsonl; exit 1; }
cat gpurun_out/r4s/panel_stream.jsonl
echo "== M=1024 GEMMs: register prefetch (6, 7) vs front-loaded reads (3)"
VARIANTS=3,6,7 CHECK_VARIANT=6 timeout -k 10 300 python scripts/bench_gemm_m1024.py > gpurun_out/r4s/gemm_m1024_rp.jsonl 2> gpurun_out/r4s/gemm_m1024_rp.err || { tail -20 gpurun_out/r4s/gemm_m1024_rp.err; exit 1; }
cat gpurun_out/r4s/gemm_m1024_rp.jsonl
echo "== bf16 MLP step, forward GEMMs on 3 / 6 / 7 (interleaved)"
for rep in 1 2; do
for v in 0 6 7; do
  DGT_GEMM_VARIANT=$v timeout -k 10 200 python bench.py --model mlp --steps 100 --warmup 10 --no-sweep > gpurun_out/r4s/mlp.json 2> gpurun_out/r4s/mlp.err || { tail -20 gpurun_out/r4s/mlp.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4s/mlp.json')); print('variant $v', d['value'], d['ms_per_step'], d['model_tflops'])" | tee -a gpurun_out/r4s/mlp_rp_ab.txt
done
done
echo done
echo "== self-launched 4-rank rehearsal on one card (process group on gloo: RCCL needs one device per rank)"
DGT_ALLOW_OVERSUBSCRIBE=1 timeout -k 10 400 python bench.py --gpus 4 --steps 20 --warmup 5 > gpurun_out/r4s/bench_self4.json 2> gpurun_out/r4s/bench_self4.err || { tail -30 gpurun_out/r4s/bench_self4.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4s/bench_self4.json').read().strip().splitlines()[-1]); print(d['value'], d['ranks'], d['config']['parallelism'], len(d['oneshot_xgmi_sweep']), d['config']['exchange'])"
echo done
