#!/bin/bash
# round 6, session E: A/B of the reducer launch paths on the bf16 engine MLP with forced collectives
set -o pipefail
O=gpurun_out/r6e2
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python scripts/engine_overlap_bench.py --no-force >> $O/ab.jsonl 2>>$O/ab.err || exit 1
  timeout -k 10 120 python scripts/engine_overlap_bench.py >> $O/ab.jsonl 2>>$O/ab.err || exit 1
  DGT_REDUCER_NATIVE=0 timeout -k 10 120 python scripts/engine_overlap_bench.py >> $O/ab.jsonl 2>>$O/ab.err || exit 1
  DGT_REDUCER_THREAD=0 timeout -k 10 120 python scripts/engine_overlap_bench.py >> $O/ab.jsonl 2>>$O/ab.err || exit 1
done
cat $O/ab.jsonl
