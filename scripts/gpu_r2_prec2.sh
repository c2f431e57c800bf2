#!/bin/bash
# Precision round 2: ALS + k-means GPU numerics tests, the rank-64 bf16 bench, fp32 ALS rank-128 and the
# certified fp32 k-means bench (vs bf16) on the BASELINE shapes.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_als_kernel.py tests/test_als_trainer.py tests/test_kmeans.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_prec.log 2>&1 || { tail -40 gpurun_out/pytest_prec.log; exit 1; }
tail -2 gpurun_out/pytest_prec.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --speed-events 0 > gpurun_out/bench64.log 2>&1 || { tail -20 gpurun_out/bench64.log; exit 1; }
echo "als64 bf16 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench64.log)"
timeout -k 10 300 python bench.py --rank-k 128 --precision fp32 --steps 10 --warmup 3 --speed-events 0 > gpurun_out/bench128_fp32.log 2>&1 || { tail -20 gpurun_out/bench128_fp32.log; exit 1; }
echo "als128 fp32 25M $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench128_fp32.log)"
timeout -k 10 300 python bench.py --rank-k 128 --precision bf16 --steps 10 --warmup 3 --speed-events 0 > gpurun_out/bench128_bf16.log 2>&1 || { tail -20 gpurun_out/bench128_bf16.log; exit 1; }
echo "als128 bf16 25M $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench128_bf16.log)"
timeout -k 10 400 python bench.py --preset c3 --steps 3 --warmup 1 > gpurun_out/bench_c3.log 2>&1 || { tail -20 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log
for p in fp32 bf16; do
  timeout -k 10 300 python bench_kmeans.py --steps 5 --warmup 2 --precision $p > gpurun_out/bench_km_$p.log 2>&1 || { tail -20 gpurun_out/bench_km_$p.log; exit 1; }
  tail -1 gpurun_out/bench_km_$p.log
done
