#!/bin/bash
# Long rows' partial sums beside the batched solve (default) vs before it.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_als_kernel.py tests/test_als_trainer.py tests/test_forced_collectives.py -m gpu > gpurun_out/r5_overlap_tests.log 2>&1 || { tail -30 gpurun_out/r5_overlap_tests.log; exit 1; }
tail -1 gpurun_out/r5_overlap_tests.log
run() {
  timeout -k 10 300 python -u bench.py --speed-events 0 --steps 10 --warmup 3 $2 > gpurun_out/r5_ovl_$1.json 2>gpurun_out/r5_ovl.err || { tail -20 gpurun_out/r5_ovl.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/r5_ovl_$1.json')); h=r['halfstep_ms']; print('$1', round(r['ms_per_step'],4), 'items', round(h['items_solve_ms'],4), 'users', round(h['users_solve_ms'],4), 'fails', r.get('solve_failures'))"
}
ORYX_ALS_PARTIAL_OVERLAP=0 run serial
run overlap
ORYX_ALS_PARTIAL_OVERLAP=0 run serial2
run overlap2
ORYX_ALS_PARTIAL_OVERLAP=0 run serial128 "--rank-k 128 --precision fp32 --steps 5 --warmup 2"
run overlap128 "--rank-k 128 --precision fp32 --steps 5 --warmup 2"
