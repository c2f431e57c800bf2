#!/bin/bash
# Long-row split (als_partial) threshold / segment sweep on the rank-64 bench (items half-step).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in ${SPLIT_CFGS:-default 4096,4096 8192,4096 8192,8192 16384,8192 2048,1024 2048,2048 1024,1024}; do
  if [ $cfg = default ]; then unset ORYX_ALS_SPLIT; else export ORYX_ALS_SPLIT=$cfg; fi
  timeout -k 10 300 python -u bench.py --speed-events 0 --steps 10 --warmup 3 > gpurun_out/r5_split_$cfg.json 2>gpurun_out/r5_split.err || { tail -20 gpurun_out/r5_split.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/r5_split_$cfg.json')); h=r['halfstep_ms']; print('$cfg', round(r['ms_per_step'],4), 'items', round(h['items_solve_ms'],4), 'users', round(h['users_solve_ms'],4))"
done
