#!/bin/bash
# Peer-push all-gather tests (two processes on one GPU), the multi-rank harness (now with the
# push run), then the generation phase attribution.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -s \
  tests/test_ipc_allgather.py tests/test_ipc_allreduce.py tests/test_multirank_gpu.py -m gpu \
  > gpurun_out/r5_ipc_allgather_tests.log 2>&1 || { tail -60 gpurun_out/r5_ipc_allgather_tests.log; exit 1; }
tail -5 gpurun_out/r5_ipc_allgather_tests.log
bash scripts/r5_gen_phases.sh v1
