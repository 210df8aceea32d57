#!/bin/bash
# round 6, session I (rerun on the final tree): the N > 1 bench paths rehearsed with 2 ranks on one card (gloo control plane,
# --force-secondary): headline exchange, secondary blocks and the new same-run baselines run and the
# line prints.  Rates are not xGMI rates.
set -o pipefail
O=gpurun_out/r6i2
mkdir -p $O
export TMPDIR=/tmp DGT_ALLOW_OVERSUBSCRIBE=1 DGT_BACKEND=gloo OMP_NUM_THREADS=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29611 \
  bench.py --gpus 2 --steps 2000 --warmup 200 --no-sweep --force-secondary --secondary-steps 20 --secondary-warmup 5 \
  > $O/b2.json 2> $O/b2.err || { tail -30 $O/b2.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r6i2/b2.json") if l.startswith("{")][-1])
print({k: d[k] for k in ("value", "n_gpus", "ranks", "vs_baseline", "params_consistent_across_ranks")})
print("baseline", d.get("baseline"))
for k in ("bf16_mlp", "fp32_engine_mlp", "bf16_mlp_zero1"):
    b = d.get(k, {})
    print(k, {x: b.get(x) for x in ("iters_per_s", "error", "exchange", "torch_baseline_iters_per_s", "speedup")})
print("baselines", {k: (v.get("iters_per_s"), v.get("error")) for k, v in (d.get("baselines") or {}).items()})
PY
