#!/bin/bash
# KP <= 64 solve-kernel variant sweep (ORYX_ALS_VARIANT 2 / 3 / 4 = factorisation issue
# priority 0 / 2 / 3) on the rank-64 headline, two passes.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for pass in 1 2 3; do
  for v in 3 4; do
    ORYX_ALS_VARIANT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --speed-events 0 \
      > gpurun_out/var_${v}_$pass.log 2>&1 || exit 1
    echo "pass $pass variant $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var_${v}_$pass.log)"
  done
done
