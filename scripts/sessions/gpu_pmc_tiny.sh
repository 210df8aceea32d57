#!/bin/bash
# PMC pass on the fused training kernel (one 100k-step launch inside bench.py), 8 SQ counters.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAIT_ANY -d $R/gpurun_out/pmc_tiny -o run --output-format csv -- python3 $R/bench.py --steps 100000 --warmup 1000 --no-sweep > $R/gpurun_out/pmc_tiny.log 2>&1 || { tail -5 $R/gpurun_out/pmc_tiny.log; exit 1; }
python3 - <<'PY'
import csv, glob, os
R = os.environ["GRAFT_REPO_ROOT"]
f = glob.glob(f"{R}/gpurun_out/pmc_tiny/**/*counter_collection.csv", recursive=True)
rows = [r for r in csv.DictReader(open(f[0])) if "tiny_mlp_train_kernel" in r["Kernel_Name"]]
by = {}
for r in rows:
    by.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
last = by[max(by, key=int)]  # the timed 100k-step launch
with open(f"{R}/gpurun_out/pmc_tiny_summary.txt", "w") as out:
    for k in sorted(last):
        print(f"{k:28s} {last[k]:.0f}", file=out)
print(open(f"{R}/gpurun_out/pmc_tiny_summary.txt").read())
PY
