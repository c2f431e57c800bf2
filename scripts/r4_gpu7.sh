set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_als_serving.py tests/test_als_common.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gpu_tests_serving.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r4_gpu_tests_serving.log; exit 1; }
timeout -k 10 400 python bench.py --preset c3 --emulate-world 8 --emulate-rank 0 --steps 3 --warmup 1 > gpurun_out/r4_emul_c3_w8.json 2> gpurun_out/r4_emul_c3_w8.err || exit 1
timeout -k 10 700 python -u bench_serving.py --items 20000000 --features 250 --sample-rate 1.0 --workers 1,4 --requests 200 --warmup 20 --rescorer > gpurun_out/r4_serving_rescorer.jsonl 2> gpurun_out/r4_serving_rescorer.err || exit 1
echo done
