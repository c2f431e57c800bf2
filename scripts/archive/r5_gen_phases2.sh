#!/bin/bash
# Generation phases after the start-up warm-up, the k-means final-pass change and the
# background ALS checkpoint; cProfile of the host side for k-means and RDF.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v2}
timeout -k 10 400 python -u bench_batch.py --ratings 25000000 --generations 2 > gpurun_out/r5_bb_als_$TAG.json 2> gpurun_out/r5_bb_als_$TAG.err || { tail -20 gpurun_out/r5_bb_als_$TAG.err; exit 1; }
timeout -k 10 400 python -u bench_batch.py --app kmeans --generations 2 --cprofile > gpurun_out/r5_bb_kmeans_$TAG.json 2> gpurun_out/r5_bb_kmeans_$TAG.err || { tail -20 gpurun_out/r5_bb_kmeans_$TAG.err; exit 1; }
timeout -k 10 400 python -u bench_batch.py --app rdf --generations 2 --cprofile > gpurun_out/r5_bb_rdf_$TAG.json 2> gpurun_out/r5_bb_rdf_$TAG.err || { tail -20 gpurun_out/r5_bb_rdf_$TAG.err; exit 1; }
echo done
