set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LEG=$PWD/oryx_amd/_native/ab/liboryx_kernels_legacy.so
for v in new legacy; do
  if [ $v = legacy ]; then export ORYX_KERNELS_SO=$LEG; fi
  echo "== phases64 $v"
  timeout -k 10 300 python -u scripts/als_phase_profile.py > gpurun_out/r5_phases64_$v.json 2> gpurun_out/ph.err || { tail -20 gpurun_out/ph.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5_phases64_$v.json'));[print(h, {k:round(x) for k,x in d[h]['cycles_per_batch'].items()}) for h in ('items','users')]"
  echo "== phases128 $v"
  ORYX_PROF_K=128 ORYX_PROF_PRECISION=fp32 timeout -k 10 300 python -u scripts/als_phase_profile.py > gpurun_out/r5_phases128_$v.json 2> gpurun_out/ph.err || { tail -20 gpurun_out/ph.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5_phases128_$v.json'));[print(h, {k:round(x) for k,x in d[h]['cycles_per_batch'].items()}) for h in ('items','users')]"
done
unset ORYX_KERNELS_SO
for cfg in "1 1" "2 1"; do
  set -- $cfg
  echo "== new gl nm=$1 wpe=$2"
  ORYX_ALS_GL_NM=$1 ORYX_ALS_GL_WPE=$2 timeout -k 10 300 python -u scripts/als_kernel_bench.py --reps 5 --rank-k 128 --precision fp32 2> gpurun_out/hs.err | cut -c1-400 || { tail -20 gpurun_out/hs.err; exit 1; }
done
