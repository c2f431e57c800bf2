set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_als_serving.py tests/test_native_http.py tests/test_serving_layer.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests_http.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r4_gpu_tests_http.log; exit 1; }
timeout -k 10 300 python -u scripts/serving_path_profile.py > gpurun_out/r4_serving_path_profile_1m_50.txt 2> gpurun_out/r4_serving_path_profile.err || exit 1
for t in 4 16; do
ORYX_BENCH_HTTP_THREADS=$t timeout -k 10 300 python -u bench_serving.py --items 1000000 --features 50 --workers 1,4,8 --requests 500 --warmup 50 > gpurun_out/r4_serving_1m_50_t$t.jsonl 2> gpurun_out/r4_serving_1m_50_t$t.err || exit 1
done
echo done
