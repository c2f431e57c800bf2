#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_features.py tests/test_kmeans.py tests/test_rdf.py tests/test_multirank_gpu.py -m gpu > gpurun_out/r5_csv_tests2.log 2>&1 || { tail -40 gpurun_out/r5_csv_tests2.log; exit 1; }
tail -2 gpurun_out/r5_csv_tests2.log
bash scripts/r5_gen_phases2.sh v5
