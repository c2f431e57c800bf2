#!/bin/bash
# Long-row split threshold / segment sweep (ORYX_ALS_SPLIT="thr,seg") on the rank-64 headline.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for pass in 1 2; do
  for sp in 4096,2048 3072,1536 6144,3072 8192,4096 16384,8192; do
    ORYX_ALS_SPLIT=$sp timeout -k 10 200 python bench.py --steps 20 --warmup 5 --speed-events 0 \
      > gpurun_out/split_${sp/,/_}_$pass.log 2>&1 || exit 1
    echo "pass $pass split $sp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/split_${sp/,/_}_$pass.log)"
  done
done
