#!/bin/bash
# Refresh the committed profiles: GPU tests, smoke, rank-64 / rank-128 ALS benches and their
# rocprofv3 kernel statistics.  Each GPU step has its own limit; the chain stops at a failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench64.log 2>&1 || { tail -20 gpurun_out/bench64.log; exit 1; }
tail -1 gpurun_out/bench64.log
timeout -k 10 300 python bench.py --rank-k 128 --steps 5 --warmup 2 > gpurun_out/bench128.log 2>&1 || { tail -20 gpurun_out/bench128.log; exit 1; }
tail -1 gpurun_out/bench128.log
for k in 64 128; do
  rm -rf gpurun_out/prof$k
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof$k -o run --output-format csv -- python3 bench.py --rank-k $k --steps 3 --warmup 1 > gpurun_out/prof$k.log 2>&1 || { tail -20 gpurun_out/prof$k.log; exit 1; }
done
ls gpurun_out/prof64 gpurun_out/prof128
timeout -k 10 300 python bench_kmeans.py --steps 5 --warmup 2 > gpurun_out/bench_kmeans.log 2>&1 || { tail -20 gpurun_out/bench_kmeans.log; exit 1; }
tail -1 gpurun_out/bench_kmeans.log
timeout -k 10 400 python bench_rdf.py --steps 2 --warmup 1 > gpurun_out/bench_rdf.log 2>&1 || { tail -20 gpurun_out/bench_rdf.log; exit 1; }
tail -1 gpurun_out/bench_rdf.log
rm -rf gpurun_out/prof_km gpurun_out/prof_rdf
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_km -o run --output-format csv -- python3 bench_kmeans.py --steps 3 --warmup 1 > gpurun_out/prof_km.log 2>&1 || { tail -20 gpurun_out/prof_km.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rdf -o run --output-format csv -- python3 bench_rdf.py --steps 1 --warmup 1 --speed-events 2000 > gpurun_out/prof_rdf.log 2>&1 || { tail -20 gpurun_out/prof_rdf.log; exit 1; }
ls gpurun_out/prof_km gpurun_out/prof_rdf
