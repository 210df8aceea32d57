# round 5: does the in-kernel step advance cost the bf16 MLP's flat Adam anything?  Interleaved A/B of
# the bf16 MLP bench (MLPTrainer, config #2) with the in-tree extension vs a build without the step
# ticket code (tools/build_ext.py --variant noticket -D DGT_ADAM_NO_TICKET), 3 fresh processes each.
set -o pipefail
O=${OUT:-gpurun_out/r5ab}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for arm in tree noticket; do
    lib=""; [ $arm = noticket ] && lib=build/variants/noticket/_C.so
    DGT_EXT_LIB=$lib timeout -k 10 200 python bench.py --model mlp --width 4096 --steps 200 --warmup 20 --no-sweep > $O/m.json 2> $O/m.err || { tail -20 $O/m.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/m.json').read().splitlines()[-1]); print('$arm', d['value'], round(d['ms_per_step']*1e3,1), 'us/step', d['model_tflops'])" | tee -a $O/adam_ab.txt
  done
done
echo done
