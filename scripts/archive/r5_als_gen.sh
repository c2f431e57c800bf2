#!/bin/bash
# ALS GPU tests (batch / publish paths) and two ALS generations.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v1}
timeout -k 10 400 python -u -m pytest tests/test_als_history.py tests/test_als_common.py tests/test_app_its.py tests/test_lambda_als.py tests/test_speed_batch.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r5_als_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/r5_als_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/r5_als_tests_$TAG.log
timeout -k 10 400 python -u bench_batch.py --ratings 25000000 --generations 2 > gpurun_out/r5_bb_als_$TAG.json 2> gpurun_out/r5_bb_als_$TAG.err || { tail -20 gpurun_out/r5_bb_als_$TAG.err; exit 1; }
echo done
