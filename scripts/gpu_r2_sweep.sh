#!/bin/bash
# /recommend sweep: every published (features, items, sample-rate) row at 1, 2, 4 workers,
# 500k users.  $1 = feature counts (comma list), $2 = item counts.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
F=${1:-50}
M=${2:-1000000,5000000,20000000}
timeout -k 10 1100 python -u bench_serving.py --sweep --sweep-features $F --sweep-items $M \
    --workers 1,2,4 --requests 300 --warmup 30 > gpurun_out/serving_sweep_$F.jsonl 2> gpurun_out/serving_sweep_$F.err \
  || { tail -20 gpurun_out/serving_sweep_$F.err; exit 1; }
cut -c1-260 gpurun_out/serving_sweep_$F.jsonl
