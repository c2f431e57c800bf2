#!/bin/bash
# The full GPU test suite and smoke() (what the driver runs at round end).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-v1}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5_pytest_gpu_$TAG.log 2>&1 || { echo tests failed; tail -60 gpurun_out/r5_pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/r5_pytest_gpu_$TAG.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/r5_smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/r5_smoke_$TAG.log
