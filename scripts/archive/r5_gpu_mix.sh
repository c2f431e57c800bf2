#!/bin/bash
# Serving under the TrafficUtil mix at 20M x 250 (LSH 0.3), HTTPS vs HTTP at 1M x 50, then the
# generation phases.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v3}
timeout -k 10 500 python -u bench_traffic.py --items 20000000 --users 500000 --features 250 --sample-rate 0.3 > gpurun_out/r5_traffic_20m_250_lsh03_$TAG.json 2> gpurun_out/r5_traffic20_$TAG.err || { tail -20 gpurun_out/r5_traffic20_$TAG.err; exit 1; }
timeout -k 10 300 python -u bench_serving.py --items 1000000 --users 500000 --features 50 --workers 4 --requests 3000 --warmup 200 --tls both > gpurun_out/r5_https_1m_50_$TAG.json 2> gpurun_out/r5_https_1m_50_$TAG.err || { tail -20 gpurun_out/r5_https_1m_50_$TAG.err; exit 1; }
bash scripts/r5_gen_phases2.sh $TAG
