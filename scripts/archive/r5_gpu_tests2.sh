set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -v --timeout 700 --timeout-method thread tests/test_multirank_gpu.py -m gpu > gpurun_out/r5_multirank.log 2>&1 || { grep -v "^E    *frame\|^E     *\[W" gpurun_out/r5_multirank.log | tail -80; exit 1; }
tail -3 gpurun_out/r5_multirank.log
