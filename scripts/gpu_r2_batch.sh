#!/bin/bash
# End-to-end batch generation at 25M ratings, certified k-means, serving spot rows, ALS profile.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_als_common.py tests/test_kmeans.py tests/test_als_serving.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_b.log 2>&1 || { tail -40 gpurun_out/pytest_b.log; exit 1; }
tail -2 gpurun_out/pytest_b.log
timeout -k 10 900 python -u bench_batch.py --ratings 25000000 > gpurun_out/bench_batch.log 2>&1 || { tail -20 gpurun_out/bench_batch.log; exit 1; }
tail -1 gpurun_out/bench_batch.log | cut -c1-1500
timeout -k 10 300 python bench_kmeans.py --steps 5 --warmup 2 --precision fp32 > gpurun_out/bench_km_fp32.log 2>&1 || { tail -20 gpurun_out/bench_km_fp32.log; exit 1; }
tail -1 gpurun_out/bench_km_fp32.log | cut -c1-300; grep -o '"init_ms.*' gpurun_out/bench_km_fp32.log
rm -rf gpurun_out/prof_km
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_km -o run --output-format csv -- python3 bench_kmeans.py --steps 3 --warmup 1 --precision fp32 > gpurun_out/prof_km.log 2>&1 || { tail -20 gpurun_out/prof_km.log; exit 1; }
find gpurun_out/prof_km -name "*kernel_stats.csv" | head -1 | xargs -I{} head -8 {}
timeout -k 10 600 python bench_serving.py --items 20000000 --features 250 --sample-rate 1.0 --workers 1,2,4 --requests 300 > gpurun_out/serv_250_20M_10.log 2>&1 || { tail -20 gpurun_out/serv_250_20M_10.log; exit 1; }
cut -c1-330 gpurun_out/serv_250_20M_10.log
