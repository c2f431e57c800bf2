#!/bin/bash
# H2D probe, the staged-copy test, then k-means / RDF generations (digest beside the parse,
# staged copy of the text).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v1}
timeout -k 10 300 python -u -m pytest tests/test_features.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5_feat_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/r5_feat_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/r5_feat_tests_$TAG.log
timeout -k 10 200 python -u scripts/h2d_probe.py 8 > gpurun_out/r5_h2d_$TAG.json 2>&1 || { tail -5 gpurun_out/r5_h2d_$TAG.json; exit 1; }
cat gpurun_out/r5_h2d_$TAG.json
timeout -k 10 400 python -u bench_batch.py --app kmeans --generations 2 > gpurun_out/r5_bb_kmeans_lazy_$TAG.json 2> gpurun_out/r5_bb_kmeans_lazy_$TAG.err || { tail -20 gpurun_out/r5_bb_kmeans_lazy_$TAG.err; exit 1; }
timeout -k 10 400 python -u bench_batch.py --app rdf --generations 2 > gpurun_out/r5_bb_rdf_lazy_$TAG.json 2> gpurun_out/r5_bb_rdf_lazy_$TAG.err || { tail -20 gpurun_out/r5_bb_rdf_lazy_$TAG.err; exit 1; }
echo done
