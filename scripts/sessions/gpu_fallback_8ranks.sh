#!/bin/bash
export DGT_ALLOW_OVERSUBSCRIBE=1  # ranks share the one card of the rehearsal box
# bench.py at 8 ranks on one GPU (gloo) with a corrupted exchange at step 100 on rank 1: every rank
# sees the replica divergence, the timed region re-runs on the RCCL path, one JSON line with
# ipc_fallback_reason set.
set -o pipefail
mkdir -p gpurun_out
DGT_BACKEND=gloo DGT_QUIET=1 OMP_NUM_THREADS=1 DGT_EXCHANGE_TIMEOUT_S=20 DGT_FAIL_AT=1:100:corrupt \
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 \
  --master-port=29533 bench.py --gpus 8 --steps 200 --warmup 20 > gpurun_out/fallback8.json 2> gpurun_out/fallback8.err \
  || { tail -30 gpurun_out/fallback8.err; exit 1; }
grep -c "re-running on the RCCL path" gpurun_out/fallback8.err
python -c "import json; d=json.loads([l for l in open('gpurun_out/fallback8.json') if l.startswith('{')][-1]); print(d['value'], d['config']['exchange'], d['ipc_fallback_reason'], d['params_consistent_across_ranks'], len(d['oneshot_xgmi_sweep']))"
