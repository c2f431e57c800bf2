#!/bin/bash
# One GPU-box session: tests, smoke, bench, and a rocprofv3 kernel profile.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
run() { echo "== $*" ; "$@"; }
if [[ $STEP == all || $STEP == test ]]; then
  run timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ $STEP == all || $STEP == smoke ]]; then
  run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -40 gpurun_out/smoke.log; exit 1; }
  tail -2 gpurun_out/smoke.log
fi
if [[ $STEP == all || $STEP == bench ]]; then
  run timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || { tail -40 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log
fi
if [[ $STEP == all || $STEP == prof ]]; then
  rm -rf gpurun_out/prof
  run timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof.log 2>&1 || { tail -40 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -15 {}'
fi
