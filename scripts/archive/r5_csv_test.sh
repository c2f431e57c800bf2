#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_features.py tests/test_kmeans.py tests/test_rdf.py -m gpu > gpurun_out/r5_csv_tests.log 2>&1 || { tail -40 gpurun_out/r5_csv_tests.log; exit 1; }
tail -2 gpurun_out/r5_csv_tests.log
timeout -k 10 400 python -u bench_batch.py --app kmeans --generations 2 > gpurun_out/r5_bb_kmeans_v4.json 2> gpurun_out/r5_bb_kmeans_v4.err || { tail -20 gpurun_out/r5_bb_kmeans_v4.err; exit 1; }
for b in 2 3; do
  ORYX_ALS_BATCH_BPC=$b timeout -k 10 300 python -u bench.py --speed-events 0 --steps 10 --warmup 3 > gpurun_out/r5_bpc$b.json 2>gpurun_out/r5_bpc.err || { tail -20 gpurun_out/r5_bpc.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/r5_bpc$b.json')); print('bpc $b', r['ms_per_step'], r['halfstep_ms'])"
done
ORYX_ALS_BATCH_BPC=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_als_kernel.py -m gpu -k "vs_reference" > gpurun_out/r5_bpc_tests.log 2>&1 || { tail -30 gpurun_out/r5_bpc_tests.log; exit 1; }
tail -1 gpurun_out/r5_bpc_tests.log
