#!/bin/bash
# One k-means and one RDF run of 2 generations (generation phases after a change).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v1}
timeout -k 10 400 python -u bench_batch.py --app kmeans --generations 2 > gpurun_out/r5_bb_kmeans_$TAG.json 2> gpurun_out/r5_bb_kmeans_$TAG.err || { tail -20 gpurun_out/r5_bb_kmeans_$TAG.err; exit 1; }
timeout -k 10 400 python -u bench_batch.py --app rdf --generations 2 > gpurun_out/r5_bb_rdf_$TAG.json 2> gpurun_out/r5_bb_rdf_$TAG.err || { tail -20 gpurun_out/r5_bb_rdf_$TAG.err; exit 1; }
echo done
