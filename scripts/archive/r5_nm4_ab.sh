#!/bin/bash
# Rank <= 64 solve: two rows per wave and two waves per SIMD (default) against four rows per
# wave, one 512-register wave per SIMD (no replica split: each row's LDL^T on its own lane
# group, no cross-row swaps).  ORYX_KERNELS_SO selects the -DORYX_ALS_BATCH_NM=4 build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
NM4=$PWD/oryx_amd/_native/ab/liboryx_kernels_nm4.so
for v in nm2 nm4 nm2b nm4b; do
  if [ ${v:0:3} = nm4 ]; then export ORYX_KERNELS_SO=$NM4; else unset ORYX_KERNELS_SO; fi
  timeout -k 10 300 python -u bench.py --speed-events 0 --steps 10 --warmup 3 > gpurun_out/r5_ab_$v.json 2>gpurun_out/r5_ab.err || { tail -20 gpurun_out/r5_ab.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/r5_ab_$v.json')); print('$v', round(r['ms_per_step'],4), {k:round(x,4) for k,x in r['halfstep_ms'].items()})"
done
export ORYX_KERNELS_SO=$NM4
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_als_kernel.py -m gpu > gpurun_out/r5_nm4_tests.log 2>&1 || { tail -30 gpurun_out/r5_nm4_tests.log; exit 1; }
tail -1 gpurun_out/r5_nm4_tests.log
timeout -k 10 300 python -u scripts/als_phase_profile.py > gpurun_out/r5_phases64_nm4.json 2> gpurun_out/ph.err || { tail -20 gpurun_out/ph.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5_phases64_nm4.json'));[print(h, {k[:10]:round(x) for k,x in d[h]['cycles_per_batch'].items()}) for h in ('items','users')]"
