#!/bin/bash
# GPU tests (incl. the GPU row formatter vs host bytes), headline bench with speed-layer
# phases, bench_batch at 25M, serving time-to-ready 1M x 250.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench64.log 2>&1 || { tail -20 gpurun_out/bench64.log; exit 1; }
tail -1 gpurun_out/bench64.log | cut -c1-2500
timeout -k 10 900 python -u bench_batch.py --ratings 25000000 > gpurun_out/bench_batch.log 2>&1 || { tail -20 gpurun_out/bench_batch.log; exit 1; }
tail -1 gpurun_out/bench_batch.log | cut -c1-1500
timeout -k 10 600 python -u bench_serving.py --time-to-ready --items 1000000 --users 100000 --features 250 > gpurun_out/ttr.log 2>&1 || { tail -20 gpurun_out/ttr.log; exit 1; }
tail -1 gpurun_out/ttr.log
