set -o pipefail
export ORYX_ALS_WIDE_VARIANT=2
cd $GRAFT_REPO_ROOT 2>/dev/null || cd /root/repo
for cfg in "2 0" "2 1" "1 0" "1 1"; do
  set -- $cfg
  ORYX_ALS_GL_NM=$1 ORYX_ALS_GL_HOLD=$2 timeout -k 10 200 python scripts/als_kernel_bench.py --rank-k 128 --precision fp32 --reps 5 > gpurun_out/hs128_nm$1_hold$2.json || exit 1
  ORYX_ALS_GL_NM=$1 ORYX_ALS_GL_HOLD=$2 timeout -k 10 200 python scripts/als_kernel_bench.py --rank-k 128 --precision bf16 --reps 5 > gpurun_out/hs128bf_nm$1_hold$2.json || exit 1
done
