#!/bin/bash
# Generation phase attribution (ALS 25M, k-means 12.5M x 256 k=1000, RDF 6.25M x 100), each
# with the train phase broken down (train_phase_s), two generations for the later-generation
# steady state.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v1}
timeout -k 10 400 python -u bench_batch.py --ratings 25000000 --generations 2 > gpurun_out/r5_bb_als_$TAG.json 2> gpurun_out/r5_bb_als_$TAG.err || { tail -20 gpurun_out/r5_bb_als_$TAG.err; exit 1; }
timeout -k 10 400 python -u bench_batch.py --app kmeans --generations 2 > gpurun_out/r5_bb_kmeans_$TAG.json 2> gpurun_out/r5_bb_kmeans_$TAG.err || { tail -20 gpurun_out/r5_bb_kmeans_$TAG.err; exit 1; }
timeout -k 10 400 python -u bench_batch.py --app rdf --generations 2 > gpurun_out/r5_bb_rdf_$TAG.json 2> gpurun_out/r5_bb_rdf_$TAG.err || { tail -20 gpurun_out/r5_bb_rdf_$TAG.err; exit 1; }
echo done
