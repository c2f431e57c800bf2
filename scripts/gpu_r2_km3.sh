#!/bin/bash
# k-means fp32: tiled full rescan of the flag-2 points -- GPU tests, bench, kernel table.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/km3_pytest.log 2>&1 || { tail -30 gpurun_out/km3_pytest.log; exit 1; }
tail -2 gpurun_out/km3_pytest.log
timeout -k 10 300 python bench_kmeans.py --precision fp32 --steps 5 --warmup 2 > gpurun_out/km3_fp32.log 2>&1 || { tail -20 gpurun_out/km3_fp32.log; exit 1; }
tail -1 gpurun_out/km3_fp32.log | grep -o '"ms_per_step[^,]*\|"rescored_points_per_step[^]]*'
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_km3 -o run --output-format csv -- python3 bench_kmeans.py --precision fp32 --steps 5 --warmup 2 > gpurun_out/prof_km3.log 2>&1 || { tail -20 gpurun_out/prof_km3.log; exit 1; }
head -6 gpurun_out/prof_km3/run_kernel_stats.csv | cut -c1-220
