set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_als_serving.py -m gpu -k "incrementally or lsh_candidates or sharded_index or kernel_and_batcher" > gpurun_out/r5_index_tests.log 2>&1 || { tail -40 gpurun_out/r5_index_tests.log; exit 1; }
tail -3 gpurun_out/r5_index_tests.log
timeout -k 10 800 python -u -m pytest -x -v --timeout 700 --timeout-method thread tests/test_multirank_gpu.py -m gpu > gpurun_out/r5_multirank.log 2>&1 || { tail -60 gpurun_out/r5_multirank.log; exit 1; }
tail -3 gpurun_out/r5_multirank.log
