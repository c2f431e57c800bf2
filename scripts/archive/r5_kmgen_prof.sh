#!/bin/bash
# Kernel trace of one k-means generation (where the evaluation's 0.65 s goes).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kmgen -o kmgen -- python -u bench_batch.py --app kmeans --generations 1 > gpurun_out/r5_kmgen_prof.json 2> gpurun_out/r5_kmgen_prof.err || { tail -20 gpurun_out/r5_kmgen_prof.err; exit 1; }
find gpurun_out/prof_kmgen -name "*kernel_stats.csv" | head -3
echo done
