#!/bin/bash
# Silhouette kernel: GPU tests, timing on the evaluation's shape, one k-means generation.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v1}
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5_km_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/r5_km_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/r5_km_tests_$TAG.log
timeout -k 10 200 python -u scripts/silhouette_probe.py > gpurun_out/r5_sil_$TAG.json 2>&1 || { tail -5 gpurun_out/r5_sil_$TAG.json; exit 1; }
tail -1 gpurun_out/r5_sil_$TAG.json
timeout -k 10 400 python -u bench_batch.py --app kmeans --generations 2 > gpurun_out/r5_bb_kmeans_sil_$TAG.json 2> gpurun_out/r5_bb_kmeans_sil_$TAG.err || { tail -20 gpurun_out/r5_bb_kmeans_sil_$TAG.err; exit 1; }
echo done
