#!/bin/bash
# Head kernels' db / loss reduction loads batched (8 per lane in flight): tests, MLP step vs _ab/, and
# kernel stats.
set -o pipefail
mkdir -p gpurun_out/ht
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_mlp_gemm.py tests/test_gpu_engine.py > gpurun_out/ht/pytest.log 2>&1 || { tail -30 gpurun_out/ht/pytest.log; exit 1; }
tail -1 gpurun_out/ht/pytest.log
rm -f gpurun_out/ab_mlp_tree.txt
bash scripts/gpu_ab_mlp_tree.sh && cp gpurun_out/ab_mlp_tree.txt gpurun_out/ht/
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ht/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model mlp --steps 20 --warmup 5 --no-sweep > $GRAFT_REPO_ROOT/gpurun_out/ht/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/ht/prof.log; exit 1; }
