#!/bin/bash
# Fused top-N scan + certified k-means: GPU tests, k-means fp32/bf16 benches, serving spot rows.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_als_serving.py tests/test_kmeans.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_serv.log 2>&1 || { tail -40 gpurun_out/pytest_serv.log; exit 1; }
tail -2 gpurun_out/pytest_serv.log
for p in fp32 bf16; do
  timeout -k 10 300 python bench_kmeans.py --steps 5 --warmup 2 --precision $p > gpurun_out/bench_km_$p.log 2>&1 || { tail -20 gpurun_out/bench_km_$p.log; exit 1; }
  tail -1 gpurun_out/bench_km_$p.log | cut -c1-200; grep -o '"init_ms.*' gpurun_out/bench_km_$p.log
done
timeout -k 10 400 python bench_serving.py --items 1000000 --features 50 --sample-rate 0.3 --workers 1,2,4 --requests 400 > gpurun_out/serv_50_1M_03.log 2>&1 || { tail -20 gpurun_out/serv_50_1M_03.log; exit 1; }
cut -c1-330 gpurun_out/serv_50_1M_03.log
timeout -k 10 600 python bench_serving.py --items 20000000 --features 250 --sample-rate 1.0 --workers 1,2,4 --requests 300 > gpurun_out/serv_250_20M_10.log 2>&1 || { tail -20 gpurun_out/serv_250_20M_10.log; exit 1; }
cut -c1-330 gpurun_out/serv_250_20M_10.log
