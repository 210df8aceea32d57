# round 5: the fused kernel's Adam as packed fp32 (v_pk_*; shipped) vs single fp32 ops
# (-D DGT_TINY_SCALAR_ADAM; tinyS2 also builds tiny_mlp.hip with -fno-slp-vectorize so the compiler
# does not re-pack it).  Interleaved fresh processes: long K (per-step chain) and the driver shape.
set -o pipefail
O=${OUT:-gpurun_out/r5tab}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for arm in tree tinyS2 tinyS; do
    lib=""; [ $arm != tree ] && lib=build/variants/$arm/_C.so
    DGT_EXT_LIB=$lib timeout -k 10 200 python bench.py --steps 100000 --warmup 5000 --no-sweep --no-secondary > $O/l.json 2> $O/l.err || { tail -20 $O/l.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/l.json').read().splitlines()[-1]); print('longK $arm', d['value'], round(d['ms_per_step']*1e3,4), 'us/step loss', d['mean_loss'])" | tee -a $O/tiny_adam_ab.txt
  done
done
for rep in 1 2; do
  for arm in tree tinyS2 tinyS; do
    lib=""; [ $arm != tree ] && lib=build/variants/$arm/_C.so
    DGT_EXT_LIB=$lib timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-sweep --no-secondary > $O/d.json 2> $O/d.err || { tail -20 $O/d.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/d.json').read().splitlines()[-1]); print('K20 $arm', d['value'], round(d['ms_per_step']*1e3,3), 'us/step loss', d['mean_loss'])" | tee -a $O/tiny_adam_ab.txt
  done
done
DGT_EXT_LIB=build/variants/tinyS2/_C.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tiny_mlp.py > $O/pytest_tinyS2.log 2>&1 || { tail -30 $O/pytest_tinyS2.log; exit 1; }
tail -1 $O/pytest_tinyS2.log
echo done
