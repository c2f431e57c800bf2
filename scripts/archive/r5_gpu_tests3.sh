set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
timeout -k 10 800 python -u -m pytest -x -q --timeout 700 --timeout-method thread tests/test_multirank_gpu.py -m gpu > gpurun_out/r5_multirank_$rep.log 2>&1 || { grep -v "^E    *frame\|^E     *\[W" gpurun_out/r5_multirank_$rep.log | grep -B2 -A30 "Traceback\|AssertionError" | head -80; exit 1; }
tail -1 gpurun_out/r5_multirank_$rep.log
done
