#!/bin/bash
# Serving under the TrafficUtil mix at 20M x 250, LSH 0.3 and 1.0.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v4}
for R in 0.3 1.0; do
  timeout -k 10 520 python -u bench_traffic.py --items 20000000 --users 500000 --features 250 --sample-rate $R > gpurun_out/r5_traffic_20m_250_lsh${R/./}_$TAG.json 2> gpurun_out/r5_traffic20_${R/./}_$TAG.err || { tail -20 gpurun_out/r5_traffic20_${R/./}_$TAG.err; exit 1; }
done

timeout -k 10 300 python -u bench_serving.py --items 1000000 --users 500000 --features 50 --workers 4 --requests 3000 --warmup 200 --tls both > gpurun_out/r5_https_1m_50_$TAG.json 2> gpurun_out/r5_https_1m_50_$TAG.err || { tail -20 gpurun_out/r5_https_1m_50_$TAG.err; exit 1; }
echo done
