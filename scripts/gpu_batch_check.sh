#!/bin/bash
# Batched ALS kernel (variant 5): GPU numerics tests, then half-step timings vs variant 3.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_als_kernel.py -k "batched" > gpurun_out/batch_tests.log 2>&1 \
  || { tail -30 gpurun_out/batch_tests.log; exit 1; }
tail -3 gpurun_out/batch_tests.log
for v in 3 5; do
  ORYX_ALS_VARIANT=$v timeout -k 10 300 python -u scripts/als_kernel_bench.py --reps 7 \
    > gpurun_out/batch_halfstep_v$v.json 2> gpurun_out/batch_halfstep_v$v.err \
    || { tail -20 gpurun_out/batch_halfstep_v$v.err; exit 1; }
  cat gpurun_out/batch_halfstep_v$v.json
done
