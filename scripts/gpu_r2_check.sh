#!/bin/bash
# Round-2 first GPU check: GPU tests, 1-GPU benches, and the RCCL code paths at world size 1
# (ORYX_FORCE_COLLECTIVES=1: process group initialised, every collective issued).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench64.log 2>&1 || { tail -20 gpurun_out/bench64.log; exit 1; }
tail -1 gpurun_out/bench64.log
ORYX_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench64_rccl1.log 2>&1 || { tail -20 gpurun_out/bench64_rccl1.log; exit 1; }
tail -1 gpurun_out/bench64_rccl1.log
ORYX_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench_kmeans.py --steps 3 --warmup 1 --points-per-gpu 2000000 > gpurun_out/bench_km_rccl1.log 2>&1 || { tail -20 gpurun_out/bench_km_rccl1.log; exit 1; }
tail -1 gpurun_out/bench_km_rccl1.log
ORYX_FORCE_COLLECTIVES=1 timeout -k 10 300 python bench_rdf.py --steps 1 --warmup 1 --examples-per-gpu 1000000 --speed-events 1000 > gpurun_out/bench_rdf_rccl1.log 2>&1 || { tail -20 gpurun_out/bench_rdf_rccl1.log; exit 1; }
tail -1 gpurun_out/bench_rdf_rccl1.log
timeout -k 10 400 python bench.py --preset c3 --steps 3 --warmup 1 > gpurun_out/bench_c3.log 2>&1 || { tail -20 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log
