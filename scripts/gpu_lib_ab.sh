#!/bin/bash
# Same-box A/B of two kernel-library builds on bench_rdf and bench_kmeans: the in-tree library
# (new) against ab/liboryx_kernels_old.so (old), alternated so box drift hits both equally.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in 1 2; do for v in new old; do
  if [[ $v == old ]]; then export ORYX_KERNELS_SO=$PWD/ab/liboryx_kernels_old.so; else unset ORYX_KERNELS_SO; fi
  timeout -k 10 400 python bench_rdf.py --steps 3 --warmup 1 --speed-events 2000 > gpurun_out/ab_rdf_$v.log 2>&1 || { tail -20 gpurun_out/ab_rdf_$v.log; exit 1; }
  echo "rdf $v $(tail -1 gpurun_out/ab_rdf_$v.log | grep -o '"ms_per_step": [0-9.]*')"
  timeout -k 10 300 python bench_kmeans.py --steps 5 --warmup 2 > gpurun_out/ab_km_$v.log 2>&1 || { tail -20 gpurun_out/ab_km_$v.log; exit 1; }
  echo "kmeans $v $(tail -1 gpurun_out/ab_km_$v.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
