#!/bin/bash
# GPU session for the k-means and RDF benchmarks: kmeans/rdf GPU tests, both benches, and a
# rocprofv3 kernel-stats profile of each.  Every GPU step has its own limit; stops at the first
# failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "== $*" ; "$@"; }
run timeout -k 10 400 python -m pytest tests/test_kmeans.py tests/test_rdf.py -x -q -m gpu > gpurun_out/pytest_apps.log 2>&1 || { tail -40 gpurun_out/pytest_apps.log; exit 1; }
tail -2 gpurun_out/pytest_apps.log
run timeout -k 10 400 python bench_kmeans.py ${KM_ARGS:---steps 10 --warmup 3} > gpurun_out/bench_kmeans.log 2>&1 || { tail -40 gpurun_out/bench_kmeans.log; exit 1; }
ORYX_KMEANS_RT=2 timeout -k 10 400 python bench_kmeans.py --steps 10 --warmup 3 > gpurun_out/bench_kmeans_rt2.log 2>&1 || { tail -20 gpurun_out/bench_kmeans_rt2.log; exit 1; }
tail -1 gpurun_out/bench_kmeans_rt2.log
tail -1 gpurun_out/bench_kmeans.log
run timeout -k 10 600 python bench_rdf.py ${RDF_ARGS:---steps 2 --warmup 1} > gpurun_out/bench_rdf.log 2>&1 || { tail -40 gpurun_out/bench_rdf.log; exit 1; }
tail -1 gpurun_out/bench_rdf.log
rm -rf gpurun_out/prof_km gpurun_out/prof_rdf
run timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_km -o run --output-format csv -- python3 bench_kmeans.py --steps 5 --warmup 1 > gpurun_out/prof_km.log 2>&1 || { tail -40 gpurun_out/prof_km.log; exit 1; }
find gpurun_out/prof_km -name "*kernel_stats.csv" | xargs -I{} head -12 {}
run timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rdf -o run --output-format csv -- python3 bench_rdf.py --steps 1 --warmup 1 --speed-events 2000 > gpurun_out/prof_rdf.log 2>&1 || { tail -40 gpurun_out/prof_rdf.log; exit 1; }
find gpurun_out/prof_rdf -name "*kernel_stats.csv" | xargs -I{} head -14 {}
