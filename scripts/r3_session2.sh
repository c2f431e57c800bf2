#!/bin/bash
# round-3 session-2 GPU batch: IPC all-reduce test, rank-128 LDS-DMA kernel sweep
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -s \
  tests/test_ipc_allreduce.py tests/test_als_history.py > gpurun_out/ipc_tests.log 2>&1 || { tail -30 gpurun_out/ipc_tests.log; exit 1; }
tail -5 gpurun_out/ipc_tests.log
bash scripts/als_gl_sweep.sh
