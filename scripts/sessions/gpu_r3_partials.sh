#!/bin/bash
# Bias-gradient partials (dgrad colsum epilogue + head partials + one reduction) replacing the
# per-layer row sums: MLP tests, then the MLP step interleaved against the previous commit (_ab/).
set -o pipefail
mkdir -p gpurun_out/part
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_mlp_gemm.py > gpurun_out/part/pytest.log 2>&1 || { tail -30 gpurun_out/part/pytest.log; exit 1; }
tail -1 gpurun_out/part/pytest.log
rm -f gpurun_out/ab_mlp_tree.txt
bash scripts/gpu_ab_mlp_tree.sh && cp gpurun_out/ab_mlp_tree.txt gpurun_out/part/
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/part/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model mlp --steps 20 --warmup 5 --no-sweep > $GRAFT_REPO_ROOT/gpurun_out/part/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/part/prof.log; exit 1; }
