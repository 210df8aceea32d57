#!/bin/bash
# The driver's K = 20 shape only, round-2 tree vs current, 8 interleaved fresh-process runs each.
set -o pipefail
mkdir -p gpurun_out/abd
export TMPDIR=/tmp
for i in 1 2 3 4 5 6 7 8; do
  for t in r2 r3; do
    d=$([ $t = r2 ] && echo build/abr2 || echo .)
    (cd $d && timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-sweep) > gpurun_out/abd/${t}_$i.json 2> gpurun_out/abd/${t}_$i.err || { tail -5 gpurun_out/abd/${t}_$i.err; exit 1; }
  done
done
python - <<'PY'
import json, statistics
for t in ("r2", "r3"):
    v = [json.load(open(f"gpurun_out/abd/{t}_{i}.json"))["value"] for i in range(1, 9)]
    print(t, "median", round(statistics.median(v)), "min", round(min(v)), "max", round(max(v)), [round(x / 1e3) for x in v])
PY
