#!/bin/bash
# SP for the dgrad + the cacheable bf16 weight copy as defaults: MLP/GEMM/engine tests, and the MLP
# step (trainer) interleaved against the previous commit (_ab/), plus the engine MLP once each.
set -o pipefail
mkdir -p gpurun_out/sp2
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_mlp_gemm.py tests/test_gpu_engine.py > gpurun_out/sp2/pytest.log 2>&1 || { tail -30 gpurun_out/sp2/pytest.log; exit 1; }
tail -1 gpurun_out/sp2/pytest.log
rm -f gpurun_out/ab_mlp_tree.txt
bash scripts/gpu_ab_mlp_tree.sh && cp gpurun_out/ab_mlp_tree.txt gpurun_out/sp2/
for t in _ab .; do
  (cd $t && timeout -k 10 300 python bench.py --model mlp --impl dgt-engine --steps 50 --warmup 10 --no-sweep > /tmp/eng.json 2> /tmp/eng.err) || { tail -5 /tmp/eng.err; exit 1; }
  python -c "import json; d=json.load(open('/tmp/eng.json')); print('engine $t', d['value'], d['ms_per_step'])" | tee -a gpurun_out/sp2/engine.txt
done
