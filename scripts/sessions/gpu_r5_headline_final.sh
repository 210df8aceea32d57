# round 5, final tree: the fused headline at long K (per-step cost of the chain) and the driver's
# shape at 2 / 8 ranks on one card (gloo rehearsal: the IPC exchange protocol, not xGMI latency).
set -o pipefail
O=${OUT:-gpurun_out/r5hf}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20000 --warmup 100 --no-secondary --no-sweep > $O/long.json 2> $O/long.err || { tail -20 $O/long.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/long.json').read().splitlines()[-1]); print('long-K', d['value'], round(d['ms_per_step']*1e3, 4), 'us/step')" | tee -a $O/headline_final.txt
done
for n in 2 8; do
  DGT_ALLOW_OVERSUBSCRIBE=1 timeout -k 10 300 python bench.py --gpus $n --steps 20 --warmup 5 --no-secondary --no-sweep > $O/r$n.json 2> $O/r$n.err || { tail -20 $O/r$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/r$n.json').read().splitlines()[-1]); print('ranks', d['ranks'], d['value'], round(d['ms_per_step']*1e3, 3), 'us/step', d['config']['exchange'], d['params_consistent_across_ranks'])" | tee -a $O/headline_final.txt
  DGT_ALLOW_OVERSUBSCRIBE=1 timeout -k 10 300 python bench.py --gpus $n --steps 5000 --warmup 100 --no-secondary --no-sweep > $O/r$n.json 2> $O/r$n.err || { tail -20 $O/r$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/r$n.json').read().splitlines()[-1]); print('ranks', d['ranks'], 'long-K', d['value'], round(d['ms_per_step']*1e3, 3), 'us/step', d['config']['exchange'], d['params_consistent_across_ranks'])" | tee -a $O/headline_final.txt
done
echo done
