set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_als_kernel.py -m gpu -k "test_kernel_vs_reference" > gpurun_out/r5_kt_new.log 2>&1
tail -15 gpurun_out/r5_kt_new.log | cut -c1-200
ORYX_KERNELS_SO=$PWD/oryx_amd/_native/ab/liboryx_kernels_legacy.so timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_als_kernel.py -m gpu -k "test_kernel_vs_reference" > gpurun_out/r5_kt_legacy.log 2>&1
tail -15 gpurun_out/r5_kt_legacy.log | cut -c1-200
