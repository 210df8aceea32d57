# round 5: the 4-wave 256x256 bf16 GEMM (variant 9: accumulators pinned in AGPRs by inline-asm MFMAs)
# -- bitwise tests against variant 8, then hot A/B vs 8 and hipBLASLt at 4096^3, 8192^3 and the MLP's
# wgrad 4096x4096x1024 (scripts/bench_gemm256_ab.py).
set -o pipefail
O=${OUT:-gpurun_out/r5w4}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_gemm.py -k "four_wave or cross_phase or identity" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VARIANTS=8,9 REPS=2 timeout -k 10 300 python scripts/bench_gemm256_ab.py > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
echo done
