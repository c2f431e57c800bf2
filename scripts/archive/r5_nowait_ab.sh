#!/bin/bash
# Rank-64 solve with and without the (disabled-by-default) long-row overlap hooks compiled in
# (-DORYX_ALS_NO_PART_WAIT=1 build in ORYX_KERNELS_SO), alternating on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
NW=$PWD/oryx_amd/_native/ab/liboryx_kernels_nowait.so
for v in def nw def2 nw2; do
  if [ ${v:0:2} = nw ]; then export ORYX_KERNELS_SO=$NW; else unset ORYX_KERNELS_SO; fi
  timeout -k 10 300 python -u bench.py --speed-events 0 --steps 20 --warmup 3 > gpurun_out/r5_nw_$v.json 2>gpurun_out/r5_nw.err || { tail -20 gpurun_out/r5_nw.err; exit 1; }
  python -c "import json; r=json.loads(open('gpurun_out/r5_nw_$v.json').read().strip().splitlines()[-1]); print('$v', round(r['ms_per_step'],4), {k:round(x,4) for k,x in r['halfstep_ms'].items()})"
done
echo done
