#!/bin/bash
# round-3 session-2 GPU batch 2: GL kernel as the default for rank > 64 / fp32
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/gpu.sh tests=als_kernel bench=--rank-k,128,--precision,fp32 bench=--rank-k,128,--precision,bf16 bench=--precision,fp32 || exit 1
ORYX_ALS_WIDE_VARIANT=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --precision fp32 > gpurun_out/bench64_fp32_wide0.json 2> gpurun_out/bench64_fp32_wide0.err || exit 1
tail -1 gpurun_out/bench64_fp32_wide0.json | cut -c1-300
ORYX_PROF_K=128 ORYX_PROF_PRECISION=fp32 bash scripts/gpu.sh phases && mv gpurun_out/phases_vdefault.json gpurun_out/phases128_fp32_nm1_v2.json
