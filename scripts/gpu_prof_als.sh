#!/bin/bash
# ALS profiling session: rank-128 bench, rocprofv3 kernel stats of the rank-64 bench, and one
# PMC pass (SQ counters) over a short run.  Every GPU step has its own time limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --rank-k 128 --steps 3 --warmup 1 > gpurun_out/b128.log 2>&1 || { tail -20 gpurun_out/b128.log; exit 1; }
tail -1 gpurun_out/b128.log
rm -rf gpurun_out/prof64
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof64.log 2>&1 || { tail -20 gpurun_out/prof64.log; exit 1; }
f=$(find gpurun_out/prof64 -name "*kernel_stats.csv" | head -1); cut -c1-200 "$f" | head -12
rm -rf gpurun_out/pmc64
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/pmc64 -o run --output-format csv -- python3 scripts/als_kernel_bench.py --reps 1 > gpurun_out/pmc64.log 2>&1 || { tail -20 gpurun_out/pmc64.log; exit 1; }
ls -R gpurun_out/pmc64 | head
