#!/bin/bash
# k-means assign A/B on one GPU: kernel tests, then bench_kmeans for each ORYX_KMEANS_RT
# setting (0 = 64-point B-operand kernel, 2 = 32-point A-operand kernel) and a kernel-trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_km.log 2>&1 || { tail -30 gpurun_out/t_km.log; exit 1; }
tail -2 gpurun_out/t_km.log
for v in ${RTS:-0 2}; do
  ORYX_KMEANS_RT=$v timeout -k 10 300 python bench_kmeans.py --steps 5 --warmup 2 > gpurun_out/bkm$v.log 2>&1 || { tail -30 gpurun_out/bkm$v.log; exit 1; }
  tail -1 gpurun_out/bkm$v.log
done
if [[ ${PROF:-1} == 1 ]]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_km -o km --output-format csv -- python3 bench_kmeans.py --steps 3 --warmup 1 > gpurun_out/prof_km.log 2>&1 || { tail -30 gpurun_out/prof_km.log; exit 1; }
  find gpurun_out/prof_km -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/km_kernel_stats.csv
  head -8 gpurun_out/km_kernel_stats.csv
fi
