set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_als_kernel.py -m gpu > gpurun_out/r5_als_kernel_tests.log 2>&1 || { tail -40 gpurun_out/r5_als_kernel_tests.log; exit 1; }
tail -3 gpurun_out/r5_als_kernel_tests.log
for v in new legacy; do
  if [ $v = legacy ]; then export ORYX_KERNELS_SO=$PWD/oryx_amd/_native/ab/liboryx_kernels_legacy.so; fi
  for a in "--rank-k 64" "--rank-k 128 --precision fp32" "--rank-k 128 --precision bf16"; do
    echo "== $v $a"
    timeout -k 10 300 python -u scripts/als_kernel_bench.py --reps 5 $a 2> gpurun_out/hs.err | cut -c1-400 || { tail -20 gpurun_out/hs.err; exit 1; }
  done
done
