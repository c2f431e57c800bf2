set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_als_serving.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests_serving.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r4_gpu_tests_serving.log; exit 1; }
timeout -k 10 600 python -u bench_serving.py --workers 1,4,8 > gpurun_out/r4_serving_1m_50_v2.jsonl 2> gpurun_out/r4_serving_1m_50_v2.err || exit 1
echo done
