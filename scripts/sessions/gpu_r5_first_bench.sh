# round 5: is the first driver-shape bench after a long GPU session slower?  (Gates v3 and v5 read
# ~504k on their first bench process after pytest + smoke, ~595-613k on the next ones.)
# Heavy GPU load for ~60 s (the bf16 MLP bench), then smoke(), then fresh bench processes with the
# timed-region breakdown; SCLK/MCLK read with rocm-smi around them.
set -o pipefail
O=${OUT:-gpurun_out/r5fb}
mkdir -p $O
export TMPDIR=/tmp
clk() { rocm-smi --showclocks 2>/dev/null | grep -E "sclk|mclk|fclk" | head -4 | tr -s ' ' | sed "s/^/[$1] /" >> $O/clocks.txt || true; }
clk idle
if [ -n "$FULL_SUITE" ]; then  # the gate's own load: the whole GPU suite in one process
  timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
else
  timeout -k 10 200 python bench.py --model mlp --width 4096 --steps 6000 --warmup 20 --no-sweep --no-secondary > $O/load.json 2> $O/load.err || { tail -20 $O/load.err; exit 1; }
fi
clk after_load
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
for i in 1 2 3 4 5 6; do
  DGT_BENCH_BREAKDOWN=1 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary > $O/b.json 2> $O/b_$i.err || { tail -20 $O/b_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('run $i', d['value'], d['ms_per_step'])" | tee -a $O/first_bench.txt
  grep "timed region" $O/b_$i.err | tee -a $O/first_bench.txt
  clk after_bench$i
done
echo done
