#!/bin/bash
# round 6 gate: what the driver runs at round end -- the GPU suite in one process, smoke(), the bench
# in the driver's shape (3 fresh processes) -- plus a kernel-stats profile of the driver's bench.
set -o pipefail
O=gpurun_out/${GATE:-r6gate}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
grep "smoke ok" $O/smoke.log
for i in 1 2 3; do
  t0=$(date +%s.%N)
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 1; }
  echo "bench wall $(python -c "import time; print(round(time.time() - $t0, 1))") s"
  python - $O/bench_$i.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(d["value"], d["vs_baseline"], d["baseline"]["iters_per_s"], "bf16", d["bf16_mlp"]["iters_per_s"], d["bf16_mlp"].get("speedup"),
      "fp32", d["fp32_engine_mlp"]["iters_per_s"], d["fp32_engine_mlp"].get("speedup"))
PY
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.out 2> $GRAFT_REPO_ROOT/$O/prof.err \
  || { tail -20 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT
head -25 $(find $O/prof -name "*kernel_stats.csv" | head -1) | cut -c1-160
