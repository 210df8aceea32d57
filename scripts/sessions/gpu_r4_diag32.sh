#!/bin/bash
set -o pipefail
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 200 python scripts/diag_f32_engine.py > $O/diag.txt 2>&1 || { tail -20 $O/diag.txt; exit 1; }
DGT_F32_SMALL_KGROUPS=1 timeout -k 10 200 python scripts/diag_f32_engine.py >> $O/diag.txt 2>&1 || { tail -20 $O/diag.txt; exit 1; }
grep -v amdgpu.ids $O/diag.txt
