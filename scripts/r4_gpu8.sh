set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_als_serving.py tests/test_native_http.py tests/test_serving_layer.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests_serving.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r4_gpu_tests_serving.log; exit 1; }
timeout -k 10 300 python -u bench_serving.py --items 1000000 --features 50 --workers 1,4,8 --requests 500 --warmup 50 > gpurun_out/r4_serving_1m_50.jsonl 2> gpurun_out/r4_serving_1m_50.err || exit 1
ORYX_BENCH_PYTHON_HTTP=1 timeout -k 10 300 python -u bench_serving.py --items 1000000 --features 50 --workers 1,4,8 --requests 500 --warmup 50 > gpurun_out/r4_serving_1m_50_pyhttp.jsonl 2> gpurun_out/r4_serving_1m_50_pyhttp.err || exit 1
timeout -k 10 700 python -u bench_serving.py --items 20000000 --features 250 --sample-rate 1.0 --workers 1,4 --requests 200 --warmup 20 > gpurun_out/r4_serving_20m_250_bf16.jsonl 2> gpurun_out/r4_serving_20m_250_bf16.err || exit 1
echo done
