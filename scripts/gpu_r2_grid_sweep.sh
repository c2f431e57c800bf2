#!/bin/bash
# ALS solve grid cap sweep (ORYX_ALS_MAX_BLOCKS), rank-64 headline bench, two passes.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for pass in 1 2; do
  for mb in 512 1024 2048 4096 8192; do
    ORYX_ALS_MAX_BLOCKS=$mb timeout -k 10 200 python bench.py --steps 20 --warmup 5 --speed-events 0 \
      > gpurun_out/grid_${mb}_$pass.log 2>&1 || exit 1
    echo "pass $pass blocks $mb $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/grid_${mb}_$pass.log)"
  done
done
