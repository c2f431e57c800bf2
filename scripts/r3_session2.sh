#!/bin/bash
# round-3 session-2 GPU batch: IPC all-reduce test, rank-128 LDS-DMA kernel sweep
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -s \
  tests/test_ipc_allreduce.py tests/test_als_history.py > gpurun_out/ipc_tests.log 2>&1 || { tail -30 gpurun_out/ipc_tests.log; exit 1; }
tail -5 gpurun_out/ipc_tests.log
# the one-shot all-reduce inside the ALS loop (forced collectives at world 1)
ORYX_FORCE_COLLECTIVES=1 ORYX_IPC_ALLREDUCE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 \
  > gpurun_out/bench64_forced_ipc.json 2> gpurun_out/bench64_forced_ipc.err || { tail -20 gpurun_out/bench64_forced_ipc.err; exit 1; }
tail -1 gpurun_out/bench64_forced_ipc.json | cut -c1-400
bash scripts/als_gl_sweep.sh
