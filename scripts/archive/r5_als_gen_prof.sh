#!/bin/bash
# ALS generation with cProfile (where publish_up / write_factors / parse go).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v1}
timeout -k 10 400 python -u bench_batch.py --ratings 25000000 --generations 2 --cprofile > gpurun_out/r5_bb_als_prof_$TAG.json 2> gpurun_out/r5_bb_als_prof_$TAG.err || { tail -20 gpurun_out/r5_bb_als_prof_$TAG.err; exit 1; }
echo done
