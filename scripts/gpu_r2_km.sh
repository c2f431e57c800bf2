#!/bin/bash
# k-means fp32 (certified) vs bf16 kernel tables.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for p in fp32 bf16; do
rm -rf gpurun_out/prof_km_$p
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_km_$p -o run --output-format csv -- python3 bench_kmeans.py --steps 5 --warmup 2 --precision $p > gpurun_out/prof_km_$p.log 2>&1 || { tail -20 gpurun_out/prof_km_$p.log; exit 1; }
grep '^{' gpurun_out/prof_km_$p.log | tail -1 | cut -c1-600
find gpurun_out/prof_km_$p -name "*kernel_stats.csv" | head -1 | xargs -I{} head -12 {} | cut -c1-180
done
