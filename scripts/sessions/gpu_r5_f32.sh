# round 5: exact-fp32 GEMM (csrc/gemm_f32_kernel.h) -- tests, then ours vs hipBLASLt per shape, with the
# planner's choice and with every tile configuration forced (DGT_F32_CFG)
set -o pipefail
OUT=${OUT:-gpurun_out/r5c}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_f32.py > $OUT/pytest.log 2>&1; echo "pytest rc=$?" >> $OUT/pytest.log
timeout -k 10 200 python scripts/bench_gemm_f32.py 1024x1024x1024 1024x4096x4096 4096x4096x4096 2048x2048x2048 256x4096x4096 1000x1000x1000 8192x8192x8192 > $OUT/bench.jsonl 2>&1
for c in 0 1 2 3; do DGT_F32_CFG=$c timeout -k 10 150 python scripts/bench_gemm_f32.py 1024x1024x1024 1024x4096x4096 4096x4096x4096 2048x2048x2048 > $OUT/bench_cfg$c.jsonl 2>&1; done
# A/B: the interleaved-load variant (tools/build_ext.py --variant ilv -D DGT_F32_INTERLEAVE=1)
if [ -f build/variants/ilv/_C.so ]; then
  DGT_EXT_LIB=build/variants/ilv/_C.so timeout -k 10 200 python scripts/bench_gemm_f32.py 1024x1024x1024 1024x4096x4096 4096x4096x4096 2048x2048x2048 8192x8192x8192 > $OUT/bench_ilv.jsonl 2>&1
  timeout -k 10 200 python scripts/bench_gemm_f32.py 1024x1024x1024 1024x4096x4096 4096x4096x4096 2048x2048x2048 8192x8192x8192 > $OUT/bench_base2.jsonl 2>&1
fi
