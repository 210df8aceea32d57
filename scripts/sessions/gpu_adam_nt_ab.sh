#!/bin/bash
# Fused wgrad+Adam epilogue with nontemporal optimizer-state accesses (DGT_ADAM_EPI_NT=1, default)
# vs plain (0): the bf16 MLP step, interleaved fresh-process runs, plus the kernel's own time.
set -o pipefail
mkdir -p gpurun_out/nt
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_mlp_gemm.py -k "adam or trainer or side" > gpurun_out/nt/pytest.log 2>&1 || { tail -20 gpurun_out/nt/pytest.log; exit 1; }
tail -1 gpurun_out/nt/pytest.log
for r in 1 2 3; do
  for nt in 0 1; do
    DGT_ADAM_EPI_NT=$nt timeout -k 10 300 python bench.py --model mlp --steps 50 --warmup 10 --no-sweep > gpurun_out/nt/nt${nt}_$r.json 2> gpurun_out/nt/nt${nt}_$r.err || { tail -5 gpurun_out/nt/nt${nt}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/nt/nt${nt}_$r.json')); print('nt=$nt run $r', d['value'], d['ms_per_step'])"
  done
done
cd /tmp
for nt in 0 1; do
  DGT_ADAM_EPI_NT=$nt timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/nt/prof_$nt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model mlp --steps 20 --warmup 5 --no-sweep > $GRAFT_REPO_ROOT/gpurun_out/nt/prof_$nt.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/nt/prof_$nt.log; exit 1; }
  python3 -c "
import csv
rows = list(csv.DictReader(open('$GRAFT_REPO_ROOT/gpurun_out/nt/prof_$nt/run_kernel_stats.csv')))
for r in rows:
    if 'gemm_nt_256_kernel<128>' in r['Name'] or 'gemm_nt_kernel<11' in r['Name'] or 'gemm_nt_kernel<76' in r['Name']:
        print('nt=$nt', r['Name'][:40], 'avg_us', round(float(r['AverageNs']) / 1e3, 1))
"
done
