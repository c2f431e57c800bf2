#!/bin/bash
# Counting-sort change check: k-means / RDF GPU tests, both benches, RDF kernel statistics.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py tests/test_rdf.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_sort.log 2>&1 || { tail -30 gpurun_out/pytest_sort.log; exit 1; }
tail -2 gpurun_out/pytest_sort.log
timeout -k 10 300 python bench_kmeans.py --steps 5 --warmup 2 > gpurun_out/bench_kmeans.log 2>&1 || { tail -20 gpurun_out/bench_kmeans.log; exit 1; }
tail -1 gpurun_out/bench_kmeans.log | cut -c1-300
for i in 1 2; do
timeout -k 10 400 python bench_rdf.py --steps 3 --warmup 1 > gpurun_out/bench_rdf.log 2>&1 || { tail -20 gpurun_out/bench_rdf.log; exit 1; }
tail -1 gpurun_out/bench_rdf.log | cut -c1-300
done
rm -rf gpurun_out/prof_rdf
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rdf -o run --output-format csv -- python3 bench_rdf.py --steps 1 --warmup 1 --speed-events 2000 > gpurun_out/prof_rdf.log 2>&1 || { tail -20 gpurun_out/prof_rdf.log; exit 1; }
ls gpurun_out/prof_rdf
