set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_mlp_gemm.py -k "adam" > gpurun_out/ws_tests.log 2>&1; rc=$?; tail -4 gpurun_out/ws_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/ws_tests.log | head -20; exit $rc; }
timeout -k 10 200 python scripts/bench_wgrad_adam.py > gpurun_out/ws_bench.jsonl 2>&1 || { tail -5 gpurun_out/ws_bench.jsonl; exit 1; }
cat gpurun_out/ws_bench.jsonl
for v in 0 6 0 6; do DGT_MLP_FUSED_VARIANT=$v timeout -k 10 200 python bench.py --model mlp --steps 50 --warmup 10 > gpurun_out/ws_mlp.json 2>/dev/null || exit 1; python -c "import json; d=json.loads(open('gpurun_out/ws_mlp.json').read().splitlines()[-1]); print('variant $v', d['value'], d['ms_per_step'])"; done
