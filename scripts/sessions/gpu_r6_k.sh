#!/bin/bash
# round 6, session K: kernel trace of the whole-step graph on the reference model (configs/ds_graph_fused.json)
set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/scripts/graph_variance_probe.py --steps 400 > $GRAFT_REPO_ROOT/$O/out.json 2> $GRAFT_REPO_ROOT/$O/err.txt \
  || { tail -20 $GRAFT_REPO_ROOT/$O/err.txt; exit 1; }
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r6k/trace/*kernel_trace.csv")[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-60:]
t0 = int(rows[0]["Start_Timestamp"])
prev = None
for r in rows[-25:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0
    print(f"{(s-t0)/1e3:8.2f} dur {(e-s)/1e3:6.2f} gap {gap:6.2f} q={r['Queue_Id']} {r['Kernel_Name'][:70]}")
    prev = e
PY
