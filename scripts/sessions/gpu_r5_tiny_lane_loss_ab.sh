# round 5: the fused kernel's deferred loss reduced lane-locally (one double per lane, one wave
# reduction per launch; shipped) vs a wave reduction at every ring flush (-D DGT_TINY_WAVE_LOSS).
# Interleaved fresh processes: long K and the driver shape; then the tiny-kernel and multi-rank
# GPU tests on the tree (loss oracles to 4 dp).
# (The candidate was not kept; this script documents how profiles/r5_tiny_lane_loss_ab.txt was taken.)
set -o pipefail
O=${OUT:-gpurun_out/r5tll}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for arm in tree waveloss; do
    lib=""; [ $arm != tree ] && lib=build/variants/$arm/_C.so
    DGT_EXT_LIB=$lib timeout -k 10 200 python bench.py --steps 100000 --warmup 5000 --no-sweep --no-secondary > $O/l.json 2> $O/l.err || { tail -20 $O/l.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/l.json').read().splitlines()[-1]); print('longK $arm', d['value'], round(d['ms_per_step']*1e3,4), 'us/step loss', d['mean_loss'])" | tee -a $O/tiny_lane_loss_ab.txt
  done
done
for rep in 1 2 3 4; do
  for arm in tree waveloss; do
    lib=""; [ $arm != tree ] && lib=build/variants/$arm/_C.so
    DGT_EXT_LIB=$lib timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-sweep --no-secondary > $O/d.json 2> $O/d.err || { tail -20 $O/d.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/d.json').read().splitlines()[-1]); print('K20 $arm', d['value'], round(d['ms_per_step']*1e3,3), 'us/step loss', d['mean_loss'])" | tee -a $O/tiny_lane_loss_ab.txt
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tiny_mlp.py tests/test_gpu_multiproc.py > $O/pytest_tree.log 2>&1 || { tail -30 $O/pytest_tree.log; exit 1; }
tail -1 $O/pytest_tree.log
echo done
