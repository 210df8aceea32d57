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
echo done
