#!/bin/bash
# Long rows: segment records stored + per-row reduction (default) vs fp32 atomics; segment sizes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_als_kernel.py tests/test_als_trainer.py -m gpu > gpurun_out/r5_partial_tests.log 2>&1 || { tail -30 gpurun_out/r5_partial_tests.log; exit 1; }
tail -1 gpurun_out/r5_partial_tests.log
run() {
  timeout -k 10 300 python -u bench.py --speed-events 0 --steps 10 --warmup 3 > gpurun_out/r5_pab_$1.json 2>gpurun_out/r5_pab.err || { tail -20 gpurun_out/r5_pab.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/r5_pab_$1.json')); h=r['halfstep_ms']; print('$1', round(r['ms_per_step'],4), 'items', round(h['items_solve_ms'],4), 'users', round(h['users_solve_ms'],4))"
}
ORYX_ALS_PARTIAL_ATOMIC=1 run atomic
run store
for cfg in 4096,1024 4096,512 4096,256 2048,512 8192,1024; do ORYX_ALS_SPLIT=$cfg run store_$cfg; done
ORYX_ALS_PARTIAL_ATOMIC=1 run atomic2
run store2
