#!/bin/bash
# The driver's K = 20 shape only, pre-window tree vs current, 8 interleaved fresh-process runs each.
set -o pipefail
mkdir -p gpurun_out/abw
export TMPDIR=/tmp
for i in 1 2 3 4 5 6 7 8; do
  for t in r2 r3; do
    d=$([ $t = r2 ] && echo build/abr3a || echo .)
    (cd $d && timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-sweep) > gpurun_out/abw/${t}_$i.json 2> gpurun_out/abw/${t}_$i.err || { tail -5 gpurun_out/abw/${t}_$i.err; exit 1; }
    [ $i -le 2 ] && { (cd $d && timeout -k 10 200 python bench.py --no-sweep) > gpurun_out/abw/${t}_def_$i.json 2>/dev/null || exit 1; }
  done
done
python - <<'PY'
import json, statistics
for t in ("r2", "r3"):
    v = [json.load(open(f"gpurun_out/abw/{t}_{i}.json"))["value"] for i in range(1, 9)]
    print(t, "median", round(statistics.median(v)), "min", round(min(v)), "max", round(max(v)), [round(x / 1e3) for x in v])
    print(t, "default", [json.load(open(f"gpurun_out/abw/{t}_def_{i}.json"))["ms_per_step"] * 1e3 for i in (1, 2)], "us/step")
PY
