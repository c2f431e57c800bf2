#!/bin/bash
# Headline bench (c2, 1 GPU), rank 128 fp32, and the emulated 8-GPU ranks (c2, c3) with the
# exposed-exchange estimates of the per-link push schedule.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v2}
timeout -k 10 300 python -u bench.py > gpurun_out/r5_bench64_$TAG.json 2> gpurun_out/r5_bench64_$TAG.err || { tail -20 gpurun_out/r5_bench64_$TAG.err; exit 1; }
timeout -k 10 300 python -u bench.py --rank-k 128 --precision fp32 > gpurun_out/r5_bench128_fp32_$TAG.json 2> gpurun_out/r5_bench128_fp32_$TAG.err || { tail -20 gpurun_out/r5_bench128_fp32_$TAG.err; exit 1; }
timeout -k 10 300 python -u bench.py --emulate-world 8 --emulate-rank 0 --preset c2 > gpurun_out/r5_emul_c2_w8_$TAG.json 2> gpurun_out/r5_emul_c2_w8_$TAG.err || { tail -20 gpurun_out/r5_emul_c2_w8_$TAG.err; exit 1; }
timeout -k 10 400 python -u bench.py --emulate-world 8 --emulate-rank 0 --preset c3 > gpurun_out/r5_emul_c3_w8_$TAG.json 2> gpurun_out/r5_emul_c3_w8_$TAG.err || { tail -20 gpurun_out/r5_emul_c3_w8_$TAG.err; exit 1; }
echo done
