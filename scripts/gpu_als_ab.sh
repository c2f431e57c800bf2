#!/bin/bash
# ALS kernel A/B on one GPU: correctness tests, bench for both solve kernels, per-half-step
# kernel timings and the per-phase cycle profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_als_kernel.py tests/test_als_trainer.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_als.log 2>&1 || { tail -30 gpurun_out/t_als.log; exit 1; }
tail -2 gpurun_out/t_als.log
for v in ${VARIANTS:-2 0}; do
  ORYX_ALS_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/b$v.log 2>&1 || { tail -30 gpurun_out/b$v.log; exit 1; }
  ORYX_ALS_VARIANT=$v timeout -k 10 300 python scripts/als_kernel_bench.py > gpurun_out/k$v.log 2>&1 || { tail -30 gpurun_out/k$v.log; exit 1; }
  tail -1 gpurun_out/k$v.log
done
python -c "
import json
import glob
for f in sorted(glob.glob('gpurun_out/b[0-9].log')):
    r=json.loads(open(f).read().strip().splitlines()[-1]); print(f, r['value'], r['ms_per_step'], r['solve_failures'])
"
if [[ ${PHASES:-1} == 1 ]]; then
  timeout -k 10 300 python scripts/als_phase_profile.py > gpurun_out/phase.log 2>&1 || { tail -30 gpurun_out/phase.log; exit 1; }
  tail -30 gpurun_out/phase.log
fi
