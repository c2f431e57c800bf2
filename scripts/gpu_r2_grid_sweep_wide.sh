#!/bin/bash
# ALS solve grid cap sweep (ORYX_ALS_MAX_BLOCKS) for the rank-128 fp32 wide kernel, two passes.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for pass in 1 2; do
  for mb in 256 512 1024 4096; do
    ORYX_ALS_MAX_BLOCKS=$mb timeout -k 10 200 python bench.py --rank-k 128 --precision fp32 --steps 10 \
      --warmup 3 --speed-events 0 > gpurun_out/gridw_${mb}_$pass.log 2>&1 || exit 1
    echo "pass $pass blocks $mb $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gridw_${mb}_$pass.log)"
  done
done
