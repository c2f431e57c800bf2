#!/bin/bash
# Full GPU test suite, the headline bench with the real speed-layer path, bench_batch at 25M,
# certified k-means, and a rocprofv3 kernel profile of the headline bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench64.log 2>&1 || { tail -20 gpurun_out/bench64.log; exit 1; }
tail -1 gpurun_out/bench64.log | cut -c1-2000
timeout -k 10 900 python -u bench_batch.py --ratings 25000000 > gpurun_out/bench_batch.log 2>&1 || { tail -20 gpurun_out/bench_batch.log; exit 1; }
tail -1 gpurun_out/bench_batch.log | cut -c1-1500
timeout -k 10 300 python bench_kmeans.py --steps 5 --warmup 2 --precision fp32 > gpurun_out/bench_km_fp32.log 2>&1 || { tail -20 gpurun_out/bench_km_fp32.log; exit 1; }
tail -1 gpurun_out/bench_km_fp32.log | cut -c1-300; grep -o '"init_ms.*' gpurun_out/bench_km_fp32.log
rm -rf gpurun_out/prof64
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof64.log 2>&1 || { tail -20 gpurun_out/prof64.log; exit 1; }
find gpurun_out/prof64 -name "*kernel_stats.csv" | head -1 | xargs -I{} head -12 {}
timeout -k 10 600 python -u bench_serving.py --time-to-ready --items 1000000 --users 100000 --features 250 > gpurun_out/ttr.log 2>&1 || { tail -20 gpurun_out/ttr.log; exit 1; }
tail -1 gpurun_out/ttr.log
