#!/bin/bash
# End-of-round validation: full GPU suite + smoke, the headline bench (1 GPU), one k-means and
# one RDF generation.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v1}
bash scripts/r5_gpu_full.sh $TAG || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r5_bench64_$TAG.json 2> gpurun_out/r5_bench64_$TAG.err || { tail -20 gpurun_out/r5_bench64_$TAG.err; exit 1; }
tail -1 gpurun_out/r5_bench64_$TAG.json
timeout -k 10 400 python -u bench_batch.py --app kmeans --generations 2 > gpurun_out/r5_bb_kmeans_final_$TAG.json 2> gpurun_out/r5_bb_kmeans_final_$TAG.err || { tail -20 gpurun_out/r5_bb_kmeans_final_$TAG.err; exit 1; }
timeout -k 10 400 python -u bench_batch.py --app rdf --generations 2 > gpurun_out/r5_bb_rdf_final_$TAG.json 2> gpurun_out/r5_bb_rdf_final_$TAG.err || { tail -20 gpurun_out/r5_bb_rdf_final_$TAG.err; exit 1; }
timeout -k 10 400 python -u bench_batch.py --ratings 25000000 --generations 2 > gpurun_out/r5_bb_als_final_$TAG.json 2> gpurun_out/r5_bb_als_final_$TAG.err || { tail -20 gpurun_out/r5_bb_als_final_$TAG.err; exit 1; }
echo done
