#!/bin/bash
# Same-box A/B of the fp32 deferred zeroing (amd.defer_zero_grad) on the reference model: eager and
# graph_module engine loops, interleaved, 3 rounds.
set -o pipefail
O=gpurun_out/r4dab
mkdir -p $O
export TMPDIR=/tmp
python - <<'PY'
import json
base = {"train_batch_size": 64, "gradient_accumulation_steps": 1, "fp16": {"enabled": False}, "zero_optimization": {"stage": 0}}
for name, amd in (("eager_on", {}), ("eager_off", {"defer_zero_grad": False}),
                  ("gm_on", {"graph_module": True}), ("gm_off", {"graph_module": True, "defer_zero_grad": False})):
    json.dump(dict(base, amd=amd), open(f"gpurun_out/r4dab/{name}.json", "w"))
PY
for i in 1 2 3; do
  for arm in eager_on eager_off gm_on gm_off; do
    timeout -k 10 200 python bench.py --impl dgt-engine --deepspeed-config $O/$arm.json --steps 3000 --warmup 200 --no-sweep > $O/$arm.out 2> $O/$arm.err || { tail -20 $O/$arm.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/$arm.out').read().strip().splitlines()[-1]); print('$arm', d['value'], round(d['ms_per_step']*1e3, 1), 'us/step', d['config']['impl'])" | tee -a $O/ab.txt
  done
done
