#!/bin/bash
# Feature-parse GPU tests, then k-means / RDF generations.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v1}
timeout -k 10 300 python -u -m pytest tests/test_features.py tests/test_kmeans.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5_feat_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/r5_feat_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/r5_feat_tests_$TAG.log
bash scripts/r5_gen_km.sh $TAG
