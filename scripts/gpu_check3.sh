#!/bin/bash
# IPC exchange session: multi-rank rehearsal tests (2 ranks on one GPU) + 2-rank benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest gpu multiproc"; timeout -k 10 600 python -m pytest tests/test_gpu_multiproc.py -x -q -m gpu -s > gpurun_out/pytest_mp.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_mp.log; [ $rc -eq 0 ] || exit $rc
echo "== bench 2 ranks"; DGT_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29517 bench.py --gpus 2 --steps 100000 --warmup 5000 > gpurun_out/bench_2r.json 2> gpurun_out/bench_2r.err || { tail -20 gpurun_out/bench_2r.err; exit 1; }
cat gpurun_out/bench_2r.json
