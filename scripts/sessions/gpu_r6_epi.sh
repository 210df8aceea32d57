#!/bin/bash
# round 6: staged-epilogue prefetch A/B -- the previous commit's extension (head), bias + mask loads
# issued ahead of the K loop (new), mask loads batched at the epilogue instead (latemask); per
# product (alternating processes) and in the bf16 MLP step.
set -o pipefail
O=gpurun_out/r6epi
mkdir -p $O
export TMPDIR=/tmp
lib() { case $1 in head) echo build/variants/head/_C.so;; latemask) echo build/variants/latemask/_C.so;; *) echo "";; esac; }
for rep in 1 2 3; do
  for ext in head new latemask; do
    DGT_EXT_LIB=$(lib $ext) timeout -k 10 120 python scripts/gemm_epi_ab.py >> $O/prod.jsonl 2> $O/prod.err || { tail -20 $O/prod.err; exit 1; }
  done
done
grep -v amdgpu $O/prod.jsonl
for rep in 1 2; do
  for ext in head new latemask; do
    DGT_EXT_LIB=$(lib $ext) timeout -k 10 200 python bench.py --model mlp --steps 300 --warmup 30 --no-sweep --no-secondary --no-baselines > $O/mlp_${ext}_$rep.json 2> $O/mlp_${ext}_$rep.err \
      || { tail -20 $O/mlp_${ext}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('mlp $ext', d['value'], d['ms_per_step'])" $O/mlp_${ext}_$rep.json
  done
done
