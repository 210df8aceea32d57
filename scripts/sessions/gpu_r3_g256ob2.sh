#!/bin/bash
# The one-barrier 256x256 kernel as the only form: GEMM tests, isolated timings vs hipBLASLt, and the
# MLP step interleaved against the previous commit (_ab/, two barriers per phase).
set -o pipefail
mkdir -p gpurun_out/ob2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_mlp_gemm.py > gpurun_out/ob2/pytest.log 2>&1 || { tail -30 gpurun_out/ob2/pytest.log; exit 1; }
tail -1 gpurun_out/ob2/pytest.log
timeout -k 10 300 python scripts/bench_gemm256_ab.py > gpurun_out/ob2/ab.jsonl 2> gpurun_out/ob2/ab.err || { tail -20 gpurun_out/ob2/ab.err; exit 1; }
cat gpurun_out/ob2/ab.jsonl
rm -f gpurun_out/ab_mlp_tree.txt
bash scripts/gpu_ab_mlp_tree.sh && cp gpurun_out/ab_mlp_tree.txt gpurun_out/ob2/
