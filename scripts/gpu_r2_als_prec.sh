#!/bin/bash
# ALS precision changes: GPU numerics tests, then a same-box A/B of the exact-c kernels
# (in-tree) against ab/liboryx_kernels_noexact.so (c_i * y_i rounded to bf16), and the c3
# preset in fp32 factor mode.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_als_kernel.py tests/test_als_trainer.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_als.log 2>&1 || { tail -30 gpurun_out/pytest_als.log; exit 1; }
tail -2 gpurun_out/pytest_als.log
for i in 1 2; do for v in new old; do
  if [[ $v == old ]]; then export ORYX_KERNELS_SO=$PWD/ab/liboryx_kernels_noexact.so; else unset ORYX_KERNELS_SO; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --speed-events 0 > gpurun_out/ab_als_$v.log 2>&1 || { tail -20 gpurun_out/ab_als_$v.log; exit 1; }
  echo "als64 $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_als_$v.log)"
done; done
unset ORYX_KERNELS_SO
timeout -k 10 300 python bench.py --rank-k 128 --precision fp32 --steps 10 --warmup 3 --speed-events 0 > gpurun_out/bench128_fp32.log 2>&1 || { tail -20 gpurun_out/bench128_fp32.log; exit 1; }
echo "als128 fp32 25M $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench128_fp32.log)"
timeout -k 10 300 python bench.py --rank-k 128 --precision bf16 --steps 10 --warmup 3 --speed-events 0 > gpurun_out/bench128_bf16.log 2>&1 || { tail -20 gpurun_out/bench128_bf16.log; exit 1; }
echo "als128 bf16 25M $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench128_bf16.log)"
timeout -k 10 400 python bench.py --preset c3 --steps 3 --warmup 1 > gpurun_out/bench_c3.log 2>&1 || { tail -20 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log
