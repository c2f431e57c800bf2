#!/bin/bash
# ALS kernel tests (default build, every rank), per-phase cycle profiles of the current rank-64
# and rank-128 fp32 solves, and two bench runs (run-to-run spread).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_als_kernel.py -m gpu > gpurun_out/r5_als_kernel_tests2.log 2>&1 || { tail -40 gpurun_out/r5_als_kernel_tests2.log; exit 1; }
tail -2 gpurun_out/r5_als_kernel_tests2.log
timeout -k 10 300 python -u scripts/als_phase_profile.py > gpurun_out/r5_phases64_now.json 2> gpurun_out/r5_phases64_now.err || { tail -20 gpurun_out/r5_phases64_now.err; exit 1; }
ORYX_PROF_K=128 ORYX_PROF_PRECISION=fp32 timeout -k 10 300 python -u scripts/als_phase_profile.py > gpurun_out/r5_phases128_now.json 2> gpurun_out/r5_phases128_now.err || { tail -20 gpurun_out/r5_phases128_now.err; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --speed-events 0 --steps 10 --warmup 3 > gpurun_out/r5_bench64_spread$i.json 2>/dev/null || exit 1
done
echo done
