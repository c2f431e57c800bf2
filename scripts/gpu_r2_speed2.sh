#!/bin/bash
# GPU tests, headline bench (speed-layer phases), bench_batch 25M.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench64.log 2>&1 || { tail -20 gpurun_out/bench64.log; exit 1; }
tail -1 gpurun_out/bench64.log | cut -c1-2500
timeout -k 10 900 python -u bench_batch.py --ratings 25000000 > gpurun_out/bench_batch.log 2>&1 || { tail -20 gpurun_out/bench_batch.log; exit 1; }
tail -1 gpurun_out/bench_batch.log | cut -c1-1500
timeout -k 10 400 python bench_rdf.py --steps 3 --warmup 1 > gpurun_out/bench_rdf.log 2>&1 || { tail -20 gpurun_out/bench_rdf.log; exit 1; }
tail -1 gpurun_out/bench_rdf.log | cut -c1-1500
rm -rf gpurun_out/prof_rdf
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rdf -o run --output-format csv -- python3 bench_rdf.py --steps 2 --warmup 1 --speed-events 0 > gpurun_out/prof_rdf.log 2>&1 || { tail -20 gpurun_out/prof_rdf.log; exit 1; }
find gpurun_out/prof_rdf -name "*kernel_stats.csv" | head -1 | xargs -I{} head -10 {} | cut -c1-160
