#!/bin/bash
# round-3 session-2 GPU batch 4: c3 shard at rank 128 fp32; batch generations with the resident history
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --preset c3 --precision fp32 --steps 3 --warmup 1 > gpurun_out/bench_c3_fp32.json 2> gpurun_out/bench_c3_fp32.err || { tail -20 gpurun_out/bench_c3_fp32.err; exit 1; }
tail -1 gpurun_out/bench_c3_fp32.json | cut -c1-300
timeout -k 10 600 python -u bench_batch.py --ratings 25000000 --generations 3 --next-ratings 2500000 > gpurun_out/bench_batch_gen3.json 2> gpurun_out/bench_batch_gen3.err || { tail -20 gpurun_out/bench_batch_gen3.err; exit 1; }
tail -1 gpurun_out/bench_batch_gen3.json | cut -c1-600
