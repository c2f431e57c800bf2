#!/bin/bash
# round-3 session-2 GPU batch 3: issue-batching / compact-address A/B, full GPU tests, profiles
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in main b0 c1; do
  so=""; [ $v != main ] && so=oryx_amd/_native/variants/liboryx_kernels_$v.so
  for prec in fp32 bf16; do
    ORYX_KERNELS_SO=$so timeout -k 10 200 python scripts/als_kernel_bench.py --rank-k 128 --precision $prec --reps 5 > gpurun_out/ab128_${v}_$prec.json || exit 1
    echo "$v $prec $(cat gpurun_out/ab128_${v}_$prec.json | cut -c1-400)"
  done
done
bash scripts/gpu.sh tests smoke bench || exit 1
bash scripts/gpu.sh prof=als128fp32:bench.py,--steps,5,--warmup,1,--rank-k,128,--precision,fp32
